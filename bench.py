#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X batched centroidal-MPC QP engine.

Metric (BASELINE.json): centroidal QPs/sec (N=10, 13-state/12-input) at batch=4096, max|du| vs the fp64 reference.
One "step" = one cmpc_solve_batch over a batch of synthetic QPs already resident in HBM: SRBD linearisation +
condensing + pyramid stacking + batched IPM + scatter/rollout (the whole hot path, nothing skipped).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N      (one process per GPU)

Multi-GPU: the QP batch shards with no data-path collective (weak scaling, B per GPU, QP ids offset by rank so every
QP's inputs are the same whatever the sharding); gloo is used only for the start/stop barriers and the max-over-ranks
time. Rank 0 prints one JSON line. `bench.py --gpus N` (N > 1) without a launcher starts its N ranks itself, one
child process per GPU, before anything touches the GPU. `value` is the solve throughput; `value_end_to_end` repeats the
timed steps with every step's U shard copied into rank 0's GPU (the xGMI result gather of SURVEY section 8e) inside the
timed window.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))

FP64_PEAK = 78.6e12   # MI355X fp64 vector/matrix, datasheet
FP32_PEAK = 157.3e12  # MI355X fp32 vector (MI355X_MICROARCH.md chip table)
SEED = 20221125


def ipm_flops(n, iters):
    """Algorithmic FLOPs of the IPM stage for one QP: per Newton iteration one Cholesky (n^3/3) and
    two solves with the factor (2 x 2n^2); per residual evaluation one H u product (2n^2)."""
    n = n.astype(np.float64)
    it = iters.astype(np.float64)
    return it * (n ** 3 / 3.0 + 4.0 * n ** 2) + (it + 1.0) * 2.0 * n ** 2


def condense_flops(contact):
    """Algorithmic FLOPs of the condensing stage per QP: for every horizon node k = 1..N the dense
    contraction of the 12 force-driven state rows, 2 * 12 * m_k^2 (Bqp_k' Q_k Bqp_k), and the propagation of the m_k
    Bqp columns through the dense 13 x 13 A_k, 2 * 13 * 13 * m_k, where m_k = 3 x (stance leg-steps before node k)."""
    m = 3 * np.cumsum(contact.reshape(contact.shape[0], contact.shape[1], -1).sum(axis=2), axis=1).astype(np.float64)
    return (2.0 * 12.0 * m ** 2 + 2.0 * 13.0 * 13.0 * m).sum(axis=1)


def ocp_flops(nu, nc, nx, iters):
    """Algorithmic FLOPs of one stage-wise OCP solve: per IPM iteration the Riccati factorisation of
    every stage k (nu_k = m, nc_k = g rows, n = nx): P [B A] 2 n^2 (n+m), the symmetric [B A]'(P [B A]) and the rows'
    Gc' Sigma Gc, lower triangles, (n+m)(n+m+1)(n+g), the Cholesky of R~ + B'PB m^3/3, Ls = M_xu Lr^-T m^2 n,
    P_k = M_xx - Ls Ls' n^2 m; two Newton solves (predictor, corrector; one without rows) of 2 (2 n^2 + 3 n m + m^2
    + 2 g (n + m)) each; and one residual evaluation per iteration plus the final one,
    2 ((n+m)^2 + n (n+m) + 2 g (n+m))."""
    n = float(nx)
    f_fact = f_solve = f_res = 0.0
    for k, m in enumerate(nu):
        m = float(m)
        g = float(nc[k]) if nc is not None else 0.0
        f_fact += 2 * n * n * (n + m) + (n + m) * (n + m + 1) * (n + g) + m ** 3 / 3 + m * m * n + n * n * m
        f_solve += 2 * (2 * n * n + 3 * n * m + m * m + 2 * g * (n + m))
        f_res += 2 * ((n + m) ** 2 + n * (n + m) + 2 * g * (n + m))
    rows = nc is not None and sum(nc) > 0
    return iters * (f_fact + (2 if rows else 1) * f_solve + f_res) + f_res


def ocp_main(args):
    """--ocp projected|rows: the HpipmInterface::solve path at the ocs2_legged_robot size (cheeta_mpc/ocp.py:
    nx = 24, 67 intervals + 3 event nodes; projected: nu 10 / 12 / 0 and no rows, the robot's own setting
    projectStateInputEqualityConstraints = true; rows: nu = 24 and 12-14 equality rows per node). One step = one
    cmpc_ocp_solve of --batch problems already resident in HBM. Reports solves/s, ms per solve at B = 1 (the MPC tick's
    latency, task.info:108: 50 Hz = 20 ms), the kernel's roofline and the CPU oracle on the host cores."""
    import ctypes as C
    import cheeta_mpc as cm
    from cheeta_mpc import ocp as gen
    from cheeta_mpc.shard import Dist
    dist = Dist()
    world, rank = dist.world, dist.rank
    ndev = cm.device_count()
    if ndev <= 0:
        raise RuntimeError("bench.py: no HIP device visible")
    cm._hchk(cm.hip().hipSetDevice(dist.local_rank % ndev), "hipSetDevice")
    n_dev, dev_ids = device_census(dist, cm.device_pci_id(dist.local_rank % ndev), args.allow_shared)
    projected = args.ocp == "projected"
    B = args.batch
    H = cm.hip()
    distinct = 16
    ps = [gen.legged_problem(7000 + rank * distinct + i, projected=projected) for i in range(distinct)]
    p0 = ps[0]
    packed = [gen.pack(p) for p in ps]
    idx = np.arange(B) % distinct
    x0 = np.array([ps[i]["x0"] for i in idx])
    recs = np.array([packed[i][0] for i in idx])
    crecs = np.array([packed[i][1] for i in idx]) if not projected else None
    solver = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=max(B, 1))
    dx0, drec = cm.DeviceArray.from_host(x0), cm.DeviceArray.from_host(recs)
    dcrec = cm.DeviceArray.from_host(crecs) if crecs is not None else None
    dx = cm.DeviceArray((B, p0["N"] + 1, p0["nx"]), np.float64)
    du = cm.DeviceArray((B, max(solver.nU, 1)), np.float64)
    dst, dit = cm.DeviceArray((B,), np.int32), cm.DeviceArray((B,), np.int32)
    stream = C.c_void_p()
    H.hipStreamCreate(C.byref(stream))
    ev = [C.c_void_p(), C.c_void_p()]
    for e in ev:
        H.hipEventCreate(C.byref(e))

    def solve(nb):
        solver.solve_device(nb, dx0, drec, dcrec, dx, du, dst, dit, stream)

    for _ in range(args.warmup):
        solve(B)
    H.hipStreamSynchronize(stream)
    dist.barrier()
    t0 = time.perf_counter()
    H.hipEventRecord(ev[0], stream)
    for _ in range(args.steps):
        solve(B)
    H.hipEventRecord(ev[1], stream)
    H.hipStreamSynchronize(stream)
    t1 = time.perf_counter()
    dist.barrier()
    elapsed = dist.max(t1 - t0)
    ms_ev = C.c_float()
    H.hipEventElapsedTime(C.byref(ms_ev), ev[0], ev[1])
    kernel_ms = ms_ev.value / args.steps  # one k_ocp_ipm launch per step on this stream
    st, it = dst.host(), dit.host()
    # B = 1: the latency of one HpipmInterface::solve on the device (kernel only, then with the host copies)
    reps = 50
    H.hipEventRecord(ev[0], stream)
    for _ in range(reps):
        solve(1)
    H.hipEventRecord(ev[1], stream)
    H.hipStreamSynchronize(stream)
    H.hipEventElapsedTime(C.byref(ms_ev), ev[0], ev[1])
    ms_b1 = ms_ev.value / reps
    t = time.perf_counter()
    for _ in range(10):
        solver.solve(x0[:1], recs[:1], crecs[:1] if crecs is not None else None)
    ms_b1_host_copy = (time.perf_counter() - t) / 10 * 1e3
    # the host path as the C++ mirror drives it: the problem written into the handle's pinned staging (no host copy),
    # cmpc_ocp_solve_host (one H2D of the records, the kernel, one D2H of x / u)
    ms_b1_host = None
    stg = solver.staging() if B == 1 else None
    if stg is not None:
        sx0, srec, screc = stg
        sx0[0] = x0[0]
        srec[0] = recs[0]
        if screc is not None:
            screc[0] = crecs[0]
        solver.solve(sx0[:1], srec[:1], screc[:1] if screc is not None else None)
        t = time.perf_counter()
        for _ in range(20):
            solver.solve(sx0[:1], srec[:1], screc[:1] if screc is not None else None)
        ms_b1_host = (time.perf_counter() - t) / 20 * 1e3
    ok = st == 0
    iters_mean = float(it[ok].mean()) if ok.any() else 0.0
    flops = sum(ocp_flops(p0["nu"], p0.get("nc"), p0["nx"], float(it[b])) for b in range(B) if ok[b])
    ach = flops / (kernel_ms * 1e-3)
    okey = f"ocp_{args.ocp}_B{B}"
    traffic, traffic_src = pmc_traffic(os.path.join(ROOT, "profiles", f"traffic_{okey}.json"), "k_ocp")
    tick = ocp_tick(gen, projected) if rank == 0 and not args.no_tick else None
    sq, sq_src = pmc_sq(okey, "k_ocp")
    sq_line = {"source": sq_src}
    if sq:
        w = sq.get("SQ_WAVE_CYCLES", 0.0)
        sq_line.update({
            "valu_active_per_wave_cycle": sq.get("SQ_ACTIVE_INST_VALU", 0.0) / w if w else None,
            "waitcnt_frac": sq.get("SQ_WAIT_ANY", 0.0) / w if w else None,
            "issue_stall_frac": sq.get("SQ_WAIT_INST_ANY", 0.0) / w if w else None,
            "valu_insts_per_wave": sq.get("SQ_INSTS_VALU", 0.0) / sq["SQ_WAVES"] if sq.get("SQ_WAVES") else None,
            "lds_bank_conflict_per_lds_inst": (sq.get("SQ_LDS_BANK_CONFLICT", 0.0) / sq["SQ_INSTS_LDS"]
                                               if sq.get("SQ_INSTS_LDS") else None)})
    value = world * B * args.steps / elapsed
    shape = (f"nx={p0['nx']}, N={p0['N']} (67 intervals + 3 event nodes), "
             + ("nu 10/12/0 projected, no rows" if projected else "nu 24/0 with 12-14 equality rows per node"))
    result = {
        "metric": f"HpipmInterface OCP-QP solves/sec (ocs2_legged_robot size: {shape}) at batch={B}",
        "value": value, "unit": "solves/s", "n_gpus": n_dev, "n_ranks": world, "shared_gpu": n_dev < world,
        "devices": dev_ids, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (cheeta_mpc/ocp.py legged_problem, 16 seeded problems tiled over the batch)",
        "config": {"workload": f"{B} OCP-QPs per GPU, {shape}, stage-wise interior-point (HPIPM's method), fp64",
                   "batch_per_gpu": B, "parallelism": f"shard{world}"},
        "ms_per_solve_b1": ms_b1, "ms_per_solve_b1_host_path": ms_b1_host,
        "ms_per_solve_b1_host_copy": ms_b1_host_copy,
        "host_path_what": ("cmpc_ocp_solve_host from Python with the problem in the handle's pinned staging (as the "
                           "C++ mirror packs it); _host_copy: from ordinary numpy arrays (one more host copy)"),
        "roofline": {"bound": "valu", "kernel": "k_ocp_ipm / k_ocp_grid", "achieved": ach / 1e12,
                     "peak": FP64_PEAK / 1e12, "unit": "TFLOP/s", "frac": ach / FP64_PEAK, "traffic": traffic,
                     "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                     "flops_per_launch": flops, "ms_per_launch": kernel_ms,
                     "flops_counted": "ocp_flops (bench.py): Riccati factorisation, Newton solves and residuals per "
                                      "IPM iteration"},
        "tick": tick,
        "sq_counters": sq_line,
        "solver": {"success_frac": float(ok.mean()), "mean_iters": iters_mean},
        "build": {"version": cm.lib().cmpc_version().decode(), "lib_md5": lib_md5()},
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py as op  # test infrastructure: the CPU restatement, timed as the baseline
        op.select_build(oracle_fast_build()[0])
        share, share_why = cpu_share()
        threads = args.cpu_threads or share
        S = min(max(args.cpu_sample // 64, threads), B)  # problems per pass
        done, wall = 0, 0.0
        while True:
            t = time.perf_counter()
            xc, uc, stc, itc = op.ocp_ipm_batch(p0["N"], p0["nx"], p0["nu"], x0[:S], recs[:S], nc=p0.get("nc"),
                                                crec=crecs[:S] if crecs is not None else None, nthreads=threads)
            wall += time.perf_counter() - t
            done += S
            if wall * threads >= 10.0 or wall >= 5.0:
                break
        ug = du.host()[:S, :solver.nU]
        rel = np.abs(ug - uc).max() / max(1.0, np.abs(uc).max())
        result["cpu_baseline"] = {"value": done / wall, "unit": "solves/s", "cores": threads, "kind": "port",
                                  "cpu_share": f"{share} ({share_why})",
                                  "sample": f"first {S} problems of the batch x{done // S}, oracle/ocp_ipm.c "
                                            f"(oracle_ocp_ipm_batch, same algorithm, Cholesky Riccati) built -O3 "
                                            f"-march={oracle_fast_build()[1]}, {threads} pthreads, {wall:.2f} s wall"}
        result["max_rel_du_vs_cpu_fp64"] = float(rel)
        result["statuses_equal_cpu"] = bool(np.array_equal(stc, st[:S]))
        # the MPC tick's comparison: one problem on one CPU thread (the oracle, the reference's algorithm), ms per solve
        reps1, t1s = 0, 0.0
        while t1s < 1.0 or reps1 < 3:
            t = time.perf_counter()
            op.ocp_ipm_batch(p0["N"], p0["nx"], p0["nu"], x0[:1], recs[:1], nc=p0.get("nc"),
                             crec=crecs[:1] if crecs is not None else None, nthreads=1)
            t1s += time.perf_counter() - t
            reps1 += 1
        result["cpu_single_thread_ms_b1"] = t1s / reps1 * 1e3
        result["cpu_single_thread_sample"] = (f"problem 0 of the batch x{reps1}, oracle_ocp_ipm_batch with 1 thread, "
                                              f"{t1s:.2f} s wall")
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.close()


def ocp_tick(gen, projected, T=60, warm=5):
    """The MPC tick through the C++ HpipmInterface mirror (tests/cpp/bin/hpipm_tick): per tick resize + solve +
    getRiccatiFeedback on the legged problem with the gait advancing one dt per tick (event nodes and per-stage inputs
    shifting, t0 = 0.015 t), host times per phase and the solve's kernel time; the medians over the ticks after the
    first `warm`. None (with the reason) when the binary is not built."""
    import struct
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "tests", "cpp", "bin", "hpipm_tick")
    if not os.path.exists(exe):
        return {"error": "tests/cpp/bin/hpipm_tick not built (make -C tests/cpp)"}
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(struct.pack("<i", T))
        for t in range(T):
            p = gen.legged_problem(9000 + t, projected=projected, t0=0.015 * t)
            rec, crec = gen.pack(p)
            rows = p.get("nc") is not None
            f.write(struct.pack("<3i", p["N"], p["nx"], 1 if rows else 0))
            f.write(np.asarray(p["nu"], np.int32).tobytes())
            if rows:
                f.write(np.asarray(p["nc"], np.int32).tobytes())
            f.write(np.asarray(p["x0"], np.float64).tobytes())
            f.write(np.asarray(rec, np.float64).tobytes())
            if rows:
                f.write(np.asarray(crec, np.float64).tobytes())
        path = f.name
    try:
        r = subprocess.run([exe, path, str(warm)], capture_output=True, text=True, timeout=300)
        out = r.stdout.strip().splitlines()
        doc = json.loads(out[-1]) if out else {"error": r.stderr[-300:]}
        doc["what"] = ("HpipmInterface (C++ mirror): resize(extractSizesFromProblem) + solve + getRiccatiFeedback per "
                       "tick, the gait advancing one dt per tick; host ms, kernel ms from HIP events")
        return doc
    finally:
        os.unlink(path)


def cpu_share():
    """(threads to use, how it was decided): the CPUs this process may run on (affinity), capped by the cgroup CPU
    quota and by OMP_NUM_THREADS when the host declares its CPU share that way (the GPU box sets it to the box's
    share of the machine's cores; os.cpu_count() there reports the whole machine)."""
    n = len(os.sched_getaffinity(0))
    why = f"affinity {n}"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            qc = max(1, int(float(q) / float(per)))
            if qc < n:
                n, why = qc, f"cgroup cpu.max {qc}"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < n:
        n, why = int(omp), f"OMP_NUM_THREADS {omp}"
    return n, why


def oracle_fast_build():
    """The -O3 oracle build for this host: liboracle_fast_v4.so (x86-64-v4, AVX-512) when /proc/cpuinfo lists the v4
    feature set, else liboracle_fast.so (x86-64-v3). Returns (file name, ISA level)."""
    try:
        with open("/proc/cpuinfo") as f:
            flags = next((ln.split(":", 1)[1].split() for ln in f if ln.startswith("flags")), [])
    except OSError:
        flags = []
    v4 = {"avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl"}
    if v4.issubset(flags) and os.path.exists(os.path.join(ROOT, "oracle", "liboracle_fast_v4.so")):
        return "liboracle_fast_v4.so", "x86-64-v4"
    return "liboracle_fast.so", "x86-64-v3"


def cpu_baseline(model_n, x0, xref, foot, contact, threads, min_cpu_s=10.0, max_wall_s=5.0, riccati=False):
    """The CPU oracle (same algorithm, fp64; the -O3 build for this host's ISA level, oracle_fast_build) on a bounded
    sample of the same batch,
    repeated until it has done about min_cpu_s of thread-time (capped at max_wall_s wall): QPs/s = QPs solved / wall
    time. riccati=True times the HPIPM-style restatement instead (no condensing; Riccati Newton steps over the stages,
    same iterates)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as op  # test infrastructure: the CPU restatement, timed as the baseline
    op.select_build(oracle_fast_build()[0])
    mo = op.default_model(model_n)
    s = op.default_settings()
    done, wall, u, st = 0, 0.0, None, None
    while True:
        t0 = time.perf_counter()
        if riccati:
            u, st, _ = op.riccati_solve_batch(mo, s, x0, xref, foot, contact, nthreads=threads)
        else:
            u, _, st, _ = op.solve_batch(mo, s, x0, xref, foot, contact, nthreads=threads, want_x=False)
        wall += time.perf_counter() - t0
        done += x0.shape[0]
        if wall * threads >= min_cpu_s or wall >= max_wall_s:
            break
    return u, st, wall, done


def lib_md5():
    import hashlib
    import cheeta_mpc as cm
    with open(cm.LIB_PATH, "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


def pmc_traffic(path, prefix):
    """HBM bytes per launch of the kernels whose name contains `prefix` (a string or a tuple of strings), from the committed rocprofv3 --pmc summary
    of this workload (profiles/traffic_<workload key>.json, written by cheeta-mpc_amd/tools/pmc_traffic.py from
    separate FETCH_SIZE / WRITE_SIZE passes of this same bench command). PMC counters cannot be read inside a normal
    run, so the value comes from the profiled run; it is reported only when the summary was taken on this exact
    build of libcmpc.so (md5), else None with the reason."""
    if not path or not os.path.exists(path):
        return None, "no PMC summary for this workload"
    with open(path) as f:
        doc = json.load(f)
    if doc.get("lib_md5") and doc["lib_md5"] != lib_md5():
        return None, f"PMC summary {os.path.basename(path)} was taken on another build of libcmpc.so"
    pre = (prefix,) if isinstance(prefix, str) else tuple(prefix)
    tot = sum(v["hbm_bytes"] for k, v in doc["kernels"].items() if any(p in k for p in pre))
    return (tot if tot > 0 else None), os.path.basename(path)


def pmc_sq(wkey, prefix):
    """Per-dispatch SQ counters of the kernels whose names contain `prefix` (a string or a tuple: the counters of
    every matching kernel summed, e.g. a two-launch stage), from the committed rocprofv3 --pmc summary of this
    workload (profiles/pmc_sq_<workload key>.json, cheeta-mpc_amd/tools/pmc_summary.py), only when it was taken on
    this exact build of libcmpc.so (md5)."""
    path = os.path.join(ROOT, "profiles", f"pmc_sq_{wkey}.json")
    if not os.path.exists(path):
        return None, "no SQ PMC summary for this workload"
    with open(path) as f:
        doc = json.load(f)
    if doc.get("lib_md5") != lib_md5():
        return None, f"SQ PMC summary {os.path.basename(path)} was taken on another build of libcmpc.so"
    pre = (prefix,) if isinstance(prefix, str) else tuple(prefix)
    acc = {}
    for k, v in doc["kernels"].items():
        if any(p in k for p in pre):
            for c, x in v["counters"].items():
                acc[c] = acc.get(c, 0.0) + x
    if not acc:
        return None, f"{pre} not in {os.path.basename(path)}"
    return acc, os.path.basename(path)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """--gpus n > 1 without a launcher: one child process per rank (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set;
    each child binds GPU LOCAL_RANK), started before this process touches the GPU; no exec. Rank 0's stdout (the JSON
    line) is relayed; the other ranks' stdout goes to stderr. Returns the exit code: non-zero if any rank failed."""
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
    # rank 0's stdout is drained by a thread; a rank that fails ends the others (they would otherwise wait in the
    # rendezvous or a barrier for the gloo timeout)
    import threading
    chunks = []
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    while any(p.poll() is None for p in procs):
        if any(p.poll() not in (None, 0) for p in procs):
            time.sleep(2.0)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            break
        time.sleep(0.1)
    codes = [p.wait() for p in procs]
    reader.join()
    sys.stdout.write(b"".join(chunks).decode())
    sys.stdout.flush()
    bad = [(r, c) for r, c in enumerate(codes) if c != 0]
    if bad:
        print(f"bench.py: rank(s) failed: {bad}", file=sys.stderr)
        return 1
    return 0


def device_census(dist, my_id, allow_shared):
    """The distinct physical GPUs (PCI identities) the ranks serve. Every rank gets the same answer; a run whose ranks
    share a GPU is refused (exit 2, reason on stderr) unless --allow-shared, which labels the line shared_gpu.
    Returns (n_distinct, ids)."""
    ids = dist.gather_object(my_id)
    n = len(set(ids))
    if n < dist.world and not allow_shared:
        if dist.rank == 0:
            print(f"bench.py: --gpus {dist.world} but the ranks serve only {n} distinct GPU(s) {sorted(set(ids))}; "
                  f"refused (pass --allow-shared to measure ranks sharing a GPU, labelled shared_gpu)", file=sys.stderr)
        dist.close()
        sys.exit(2)
    return n, ids


def stub_rank(args):
    """--stub (CPU tests of the launcher): the rank set-up, device census, barriers and max-over-ranks of a real run
    over gloo, no HIP call; rank 0 prints a JSON line carrying n_gpus like the real one. --stub-fail-rank r makes rank
    r exit 3; --stub-devices a,b,.. gives rank r the PCI identity entry r (default: one distinct device per rank)."""
    sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
    from cheeta_mpc.shard import Dist
    dist = Dist()
    if dist.rank == args.stub_fail_rank:
        sys.exit(3)
    devs = args.stub_devices.split(",") if args.stub_devices else [f"0000:{r:02x}:00.0" for r in range(dist.world)]
    n_dev, ids = device_census(dist, devs[dist.rank % len(devs)], args.allow_shared)
    dist.barrier()
    t = dist.max(float(dist.rank))
    if dist.rank == 0:
        print(json.dumps({"metric": "stub", "n_gpus": n_dev, "n_ranks": dist.world, "shared_gpu": n_dev < dist.world,
                          "devices": ids, "max_rank": t, "stub": True}), flush=True)
    dist.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 200 timed steps (~0.1 s at the headline) after 50 warm-up steps; with only 3 warm-up steps the first
    # timed steps still ran at the idle clock (headline 7.93-8.10 M QPs/s at 3 / 20 against 8.38-8.45 M at 3 / 100,
    # profiles/r03_warmup_ab.txt)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    # the W warm-up steps are extended, untimed, until the GPU has run the workload for at least this long: a 5-step
    # warm-up (2.5 ms at the headline) leaves the first timed steps at the idle clock (driver's 20 / 5 command:
    # 8.14 M QPs/s against 9.11 M at 200 / 50 on the same box, profiles/r04m_bench_*.json); reported as warmup_run
    ap.add_argument("--min-warmup-s", type=float, default=0.5)
    ap.add_argument("--batch", type=int, default=4096, help="QPs per GPU per step")
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--precision", choices=["f64", "f32"], default="f64")
    ap.add_argument("--gait", type=int, default=0, help="0 trot (configs 2-4), 1 mixed trot/bound/pronk (config 5)")
    ap.add_argument("--all-stance", action="store_true",
                    help="every leg in stance at every step (pronk): n = 12 N, the largest condensed size class")
    ap.add_argument("--sqp-iters", type=int, default=0,
                    help="> 0: one step = the batched SQP on the bilinear NLP (cmpc_sqp_solve_batch), this many "
                         "SQP iterations at most; not the headline metric")
    ap.add_argument("--nlp", action="store_true",
                    help="with --sqp-iters: the reference's NLP with the later runs' footholds as decision variables "
                         "(cmpc_nlp_solve_batch) instead of frozen footholds")
    ap.add_argument("--inflight", type=int, default=1,
                    help="independent batches in flight: step i runs on context / stream i %% K (a serving pattern; "
                         "each step is still one full batch through the whole hot path). Default 1: the headline")
    ap.add_argument("--graph", type=int, choices=[0, 1], default=0,
                    help="1: each context's step is captured once into a hipGraph (stream capture of cmpc_solve_batch) "
                         "and the timed steps replay it (the stage times then come from direct steps after them)")
    ap.add_argument("--stage-events", choices=["timed", "after"], default="timed",
                    help="timed: HIP events around every stage of every timed step (the roofline's kernel times come "
                         "from the timed region itself); after: the timed steps run without events and the stage times "
                         "come from as many profiled steps run right after them")
    ap.add_argument("--event-frac", type=float, default=0.25,
                    help="with --stage-events timed: the events bracket the stages of the last this fraction of the "
                         "timed steps (each timed event costs ~1 %% of a headline step: 4 per call, 3-4 %% with "
                         "every step profiled, profiles/r03d_events_ab.txt); 1 = every timed step")
    ap.add_argument("--ric", type=int, choices=[0, 1, 2], default=0,
                    help="CMPC_PATH_RICCATI: 0 condensed, 1 stage-wise kernel for the n > 64 classes, 2 for every QP")
    ap.add_argument("--path", action="append", default=[], metavar="OPTION=VALUE",
                    help="kernel-path option of the context (cmpc_set_path; A/B runs): FUSED64, FUSED128, DIRECT or "
                         "RICCATI, e.g. --path FUSED128=1; repeatable")
    ap.add_argument("--cpu-sample", type=int, default=4096, help="QPs in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host's CPU share (cpu_share())")
    ap.add_argument("--traffic-json", default="",
                    help="PMC summary giving roofline.traffic (default: profiles/traffic_<workload key>.json)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end pass (solve + result gather timed)")
    ap.add_argument("--ocp", choices=["projected", "rows"], default="",
                    help="benchmark the HpipmInterface::solve path (cmpc_ocp_solve) on ocs2_legged_robot-size OCP-QPs "
                         "instead of the centroidal headline; --batch problems per step")
    ap.add_argument("--no-tick", action="store_true", help="--ocp: skip the C++ mirror tick line (counter passes)")
    ap.add_argument("--cadence", type=float, default=0.0, metavar="MS",
                    help="> 0: after the timed run, one step every MS milliseconds (20 = the MPC's 50 Hz, task.info:108) "
                         "for --cadence-calls calls, each synchronised; the per-call latency distribution is added to "
                         "the line as 'cadence' (the clocks a 50 Hz loop runs at, not a saturated stream)")
    ap.add_argument("--cadence-calls", type=int, default=100)
    ap.add_argument("--allow-shared", action="store_true",
                    help="let ranks share a GPU (rehearsal on a one-GPU box); the line then says shared_gpu and n_gpus "
                         "counts distinct devices")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stub-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--stub-devices", default="", help=argparse.SUPPRESS)
    args = ap.parse_args()

    ws = os.environ.get("WORLD_SIZE")
    if ws is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if ws is not None and int(ws) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws} (the launcher started a different rank count)")
    if args.stub:
        stub_rank(args)
        return
    if args.ocp:
        ocp_main(args)
        return

    import cheeta_mpc as cm
    from cheeta_mpc.shard import Dist
    dist = Dist()  # gloo barriers + max-over-ranks only; no collective on the data path
    world, rank = dist.world, dist.rank
    ndev = cm.device_count()
    if ndev <= 0:
        raise RuntimeError("bench.py: no HIP device visible")
    # one GPU per rank; the modulo covers launchers that expose only the rank's own GPU (HIP_VISIBLE_DEVICES); the
    # census refuses ranks that would share a device (one visible GPU for --gpus N > 1) unless --allow-shared
    cm._hchk(cm.hip().hipSetDevice(dist.local_rank % ndev), "hipSetDevice")
    n_dev, dev_ids = device_census(dist, cm.device_pci_id(dist.local_rank % ndev), args.allow_shared)
    barrier, max_over_ranks = dist.barrier, dist.max

    B, N = args.batch, args.horizon
    prec = cm.F64 if args.precision == "f64" else cm.F32
    model = cm.default_model(N)
    if prec == cm.F64:
        settings = cm.default_settings()
    else:
        settings = cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4)
    K = max(1, args.inflight)
    path = {cm.PATH_RICCATI: args.ric} if args.ric else {}
    for kv in args.path:
        k, v = kv.split("=")
        path[getattr(cm, "PATH_" + k.upper())] = int(v)
    path = path or None
    engs = [cm.Engine(model, settings, precision=prec, max_batch=B, path=path) for _ in range(K)]
    eng = engs[0]
    x0, xref, foot, contact = cm.generate_device(model, SEED, B, gait=args.gait, offset=rank * B)
    if args.all_stance:
        contact.upload(np.ones((B, N, 4), np.uint8))
    outs = [(cm.DeviceArray((B, N, 4, 3), np.float64), cm.DeviceArray((B,), np.int32), cm.DeviceArray((B,), np.int32))
            for _ in range(K)]
    u, st, it = outs[0]
    H = cm.hip()
    import ctypes as C
    streams = []
    for _ in range(K):
        sh = C.c_void_p()
        H.hipStreamCreate(C.byref(sh))
        streams.append(sh)
    stream = streams[0]

    sqp_qi = cm.DeviceArray((B,), np.int32)
    sqp_si = cm.DeviceArray((B,), np.int32)
    feet_out = cm.DeviceArray((B, N + 1, 4, 3), np.float64) if args.nlp else None

    def step(i):
        e, (uo, so, io), sh = engs[i % K], outs[i % K], streams[i % K]
        if args.sqp_iters > 0 and args.nlp:
            cm.lib().cmpc_nlp_solve_batch(e.ctx, B, x0.ptr, xref.ptr, foot.ptr, contact.ptr, args.sqp_iters, 1e-6,
                                          uo.ptr, feet_out.ptr, None, so.ptr, sqp_qi.ptr, sqp_si.ptr, sh)
        elif args.sqp_iters > 0:
            cm.lib().cmpc_sqp_solve_batch(e.ctx, B, x0.ptr, xref.ptr, foot.ptr, contact.ptr, args.sqp_iters, 1e-6,
                                          uo.ptr, None, so.ptr, sqp_qi.ptr, sqp_si.ptr, sh)
        else:
            e.solve_device(B, x0, xref, foot, contact, uo, None, so, io, sh)

    # value_short_warmup: the same timed loop right after 5 warm-up steps with no extension (the GPU near its idle
    # clock), before the regular warm-up below; it separates clock warm-up from kernel gains in the headline
    for i in range(5):
        step(i)
    H.hipDeviceSynchronize()
    barrier()
    t_s = time.perf_counter()
    for i in range(args.steps):
        step(i)
    H.hipDeviceSynchronize()
    value_short = world * B * args.steps / max_over_ranks(time.perf_counter() - t_s)
    for i in range(args.warmup):
        step(i)
    H.hipDeviceSynchronize()
    warmup_run = args.warmup
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < args.min_warmup_s:  # same steps, untimed, synchronised every 8 so the
        for _ in range(8):                               # condition tracks GPU time rather than the launch queue
            step(warmup_run)
            warmup_run += 1
        H.hipDeviceSynchronize()

    direct_step = step
    if args.graph and args.sqp_iters > 0:
        sys.exit("bench.py: --graph captures cmpc_solve_batch only (the SQP reads a convergence flag back per iteration)")
    if args.graph:  # one captured step per context / stream; the timed loop replays them
        for fn, at in (("hipStreamBeginCapture", [C.c_void_p, C.c_int]),
                       ("hipStreamEndCapture", [C.c_void_p, C.POINTER(C.c_void_p)]),
                       ("hipGraphInstantiate", [C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p, C.c_char_p, C.c_size_t]),
                       ("hipGraphLaunch", [C.c_void_p, C.c_void_p])):
            getattr(H, fn).argtypes = at
        exes = []
        for k in range(K):
            g, ex = C.c_void_p(), C.c_void_p()
            cm._hchk(H.hipStreamBeginCapture(streams[k], 0), "hipStreamBeginCapture")
            direct_step(k)
            cm._hchk(H.hipStreamEndCapture(streams[k], C.byref(g)), "hipStreamEndCapture")
            cm._hchk(H.hipGraphInstantiate(C.byref(ex), g, None, None, 0), "hipGraphInstantiate")
            exes.append(ex)

        def step(i):
            cm._hchk(H.hipGraphLaunch(exes[i % K], streams[i % K]), "hipGraphLaunch")
        for i in range(args.warmup):
            step(i)
        H.hipDeviceSynchronize()

    timed_events = args.stage_events == "timed" and not args.graph
    # context 0's calls in the timed loop are steps 0, K, 2K, ...; the last n_prof of them carry the stage events
    n_ctx0 = (args.steps + K - 1) // K
    n_prof = min(n_ctx0, max(1, int(np.ceil(n_ctx0 * min(max(args.event_frac, 0.0), 1.0)))))
    i_prof = (n_ctx0 - n_prof) * K
    barrier()
    H.hipDeviceSynchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if timed_events and i == i_prof:
            cm.lib().cmpc_profile_begin(eng.ctx, n_prof)
        step(i)
    for sh in streams:
        H.hipStreamSynchronize(sh)
    H.hipDeviceSynchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = max_over_ranks(t1 - t0)
    if not timed_events:  # stage times from the same number of profiled steps right after the timed ones
        cm.lib().cmpc_profile_begin(eng.ctx, (args.steps + K - 1) // K)
        for i in range(args.steps):
            direct_step(i)
        H.hipDeviceSynchronize()
    ms = [C.c_double(0), C.c_double(0), C.c_double(0)]
    ncalls = C.c_int(0)
    cm.lib().cmpc_profile_end(eng.ctx, *[C.byref(m) for m in ms], C.byref(ncalls))
    # stage 1 / 2 / 3 (cmpc.h): condensing / IPM / expand, or on the fused path fused n<=64 / bigger classes / expand
    ms_cond, ms_ipm, ms_exp = (m.value / max(ncalls.value, 1) for m in ms)

    # end-to-end pass ("xGMI only for result gather"): the same K steps with every step's U shard
    # written into rank 0's GPU right after its solve (IPC-mapped device-to-device copy on the step's stream: a peer
    # write over xGMI between GPUs; no collective), all inside the timed window. A failure is reported, not fatal.
    row = N * 12 * 8
    gather = {"what": "every step: solve, then U of the rank's shard into rank 0's GPU (cmpc_ipc_open + "
                      "cmpc_gather_shard on the step's stream), inside the timed window",
              "bytes_per_step": world * B * row, "ms_per_step": None}
    value_e2e = None
    if not args.no_e2e and args.sqp_iters <= 0:
        # ResultGather's constructor and the checks below reach every collective on every rank and raise on all ranks
        # together, so the collectives stay matched whatever fails
        try:
            from cheeta_mpc.shard import ResultGather
            rg = ResultGather(dist, world * B * row)
            try:
                for i in range(args.warmup):
                    step(i)
                    cm._chk(cm.lib().cmpc_gather_shard(rg.dst, rank * B * row, outs[i % K][0].ptr, B * row,
                                                       streams[i % K]), "cmpc_gather_shard")
                H.hipDeviceSynchronize()
                barrier()
                H.hipDeviceSynchronize()
                t0 = time.perf_counter()
                for i in range(args.steps):
                    step(i)
                    cm._chk(cm.lib().cmpc_gather_shard(rg.dst, rank * B * row, outs[i % K][0].ptr, B * row,
                                                       streams[i % K]), "cmpc_gather_shard")
                for sh in streams:
                    H.hipStreamSynchronize(sh)
                H.hipDeviceSynchronize()
                t1 = time.perf_counter()
                barrier()
                e2e = max_over_ranks(t1 - t0)
                value_e2e = world * B * args.steps / e2e
                gather["ms_per_step"] = e2e / args.steps * 1e3
                # rank 0's buffer now holds every rank's U of the last step: its own slice must equal its solve
                if rank == 0:
                    got = rg.host(np.float64, (world * B, N, 4, 3))[:B]
                    gather["rank0_slice_exact"] = bool(np.array_equal(got, outs[(args.steps - 1) % K][0].host()))
            finally:
                rg.close()
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            gather["error"] = repr(e)[:200]

    cadence = None
    if args.cadence > 0:  # one synchronised call per period, as the MPC loop issues them
        lat = []
        nxt = time.perf_counter()
        for i in range(args.cadence_calls):
            nxt += args.cadence * 1e-3
            t = time.perf_counter()
            direct_step(0)
            H.hipStreamSynchronize(stream)
            lat.append((time.perf_counter() - t) * 1e3)
            time.sleep(max(0.0, nxt - time.perf_counter()))
        lat = np.array(lat)
        cadence = {"period_ms": args.cadence, "calls": args.cadence_calls,
                   "latency_ms": {"p50": float(np.percentile(lat, 50)), "p90": float(np.percentile(lat, 90)),
                                  "p99": float(np.percentile(lat, 99)), "max": float(lat.max()),
                                  "first": float(lat[0])},
                   "what": "host time of one cmpc_solve_batch call + stream sync, one call per period"}

    status = st.host()
    iters = it.host() if args.sqp_iters <= 0 else sqp_qi.host()
    ct = contact.host()
    nvar = 3 * ct.reshape(B, -1).sum(axis=1)
    ok = status == 0
    fused = bool(cm.lib().cmpc_ctx_fused(eng.ctx)) and args.sqp_iters <= 0
    peak = FP64_PEAK if prec == cm.F64 else FP32_PEAK
    fl_ipm = ipm_flops(nvar, iters) * ok
    fl_cond = condense_flops(ct) * (nvar > 0)
    small = nvar <= 64

    headline = (B == 4096 and N == 10 and prec == cm.F64 and args.gait == 0 and not args.all_stance and K == 1)
    wkey = (f"N{N}_B{B}_{'f64' if prec == cm.F64 else 'f32'}_"
            f"{'allstance' if args.all_stance else ('trot' if args.gait == 0 else 'mixed')}")
    tpath = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{wkey}.json")
    unit_name = "fp64 VALU" if prec == cm.F64 else "fp32 VALU"

    def roof(kernel, flops, ms, bound, prefix, what):
        tr, src = pmc_traffic(tpath, prefix)
        a = flops / (ms * 1e-3) if ms > 0 else 0.0
        return {"bound": bound, "compute_unit": unit_name if bound == "valu" else "fp64/fp32 MFMA", "kernel": kernel,
                "achieved": a / 1e12, "peak": peak / 1e12, "unit": "TFLOP/s", "frac": a / peak, "traffic": tr,
                "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": src, "flops_per_launch": flops,
                "ms_per_launch": ms, "flops_counted": what}

    if fused:
        # stage 1 = k_solve64: condensing and IPM of the n <= 64 class in one launch (its algorithmic work is both
        # stages' FLOPs of those QPs); stage 2 = the bigger classes (their condensing + IPM).
        # The roofline line is the dominant (longer) stage.
        f_small = float(fl_ipm[small].sum() + fl_cond[small].sum())
        f_big = float(fl_ipm[~small].sum() + fl_cond[~small].sum())
        r_small = roof("k_solve64 (fused condensing + IPM, n<=64)", f_small, ms_cond, "valu", "k_solve64",
                       "IPM + condensing FLOPs of the n<=64 QPs")
        big_kernels = ("k_solve128", "k_srbd_condense", "k_ipm128x", "k_ipm_tiled", "k_class_lists")
        r_big = roof("bigger classes (k_solve128 or k_srbd_condense + k_ipm128x n<=128; k_srbd_condense + "
                     "k_ipm_tiled n<=256)", f_big, ms_ipm, "valu", big_kernels,
                     "IPM + condensing FLOPs of the n>64 QPs")
        roofline, other = (r_small, r_big) if ms_cond >= ms_ipm else (r_big, r_small)
        stages = {"solve64_fused": ms_cond, "bigger_classes": ms_ipm, "expand": ms_exp}
        f_all = f_small + f_big
        extra = {"roofline_other_stage": other,
                 "roofline_solve": roof("whole solve (all classes, condensing + IPM)", f_all, ms_cond + ms_ipm,
                                        "valu", "cmpc::k_", "IPM + condensing FLOPs of every QP")}
        # the condensing's H = Bqp' Q Bqp contraction runs on the matrix cores: its MFMA rate and busy fraction, for
        # the dominant stage's kernels, from the committed SQ counters of this build (executed MFMA FLOPs = MOPS x 512)
        if ms_cond >= ms_ipm:
            mk, mms, what = ("k_solve64",), ms_cond, "k_solve64 condensing phase"
        else:
            mk, mms, what = (("k_solve128",) if cm.lib().cmpc_get_path(eng.ctx, cm.PATH_FUSED128) == 1 else
                             ("k_srbd_condense",)), ms_ipm, "bigger-class condensing"
        c, src = pmc_sq(wkey, mk)
        mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F64" if prec == cm.F64 else "SQ_INSTS_VALU_MFMA_MOPS_F32") if c else None
        if mops is not None and mms > 0:
            mfl = 512.0 * mops
            cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0  # GRBM_GUI_ACTIVE sums the 8 XCDs
            extra["mfma_condensing"] = {
                "kernel": "%s (H = Bqp' Q Bqp on v_mfma_%s_16x16x4 in %s), rate over the stage's duration"
                          % (what, "f64" if prec == cm.F64 else "f32", "+".join(mk)),
                "mfma_flops_per_launch": mfl, "achieved": mfl / (mms * 1e-3) / 1e12, "peak": peak / 1e12,
                "unit": "TFLOP/s", "frac": mfl / (mms * 1e-3) / peak,
                "mfma_busy_frac": (c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0)
                                   if cyc > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in c else None),
                "source": src}
        else:
            extra["mfma_condensing"] = {"kernel": what, "achieved": None, "source": src}
    else:
        roofline = roof("IPM stage (k_ipm64 n<=64, k_ipm128x n<=128, k_ipm_tiled<16> n<=256)", float(fl_ipm.sum()),
                        ms_ipm, "valu", "k_ipm", "IPM FLOPs")
        stages = {"condense": ms_cond, "ipm": ms_ipm, "expand": ms_exp}
        # the condensing stage's Bqp' Q Bqp contraction runs on MFMA (v_mfma_f64_16x16x4 / f32_16x16x4)
        extra = {"roofline_condense": roof("condensing stage (k_condense64 / k_srbd_condense)", float(fl_cond.sum()),
                                           ms_cond, "mfma", "condense", "condensing FLOPs")}

    value = world * B * args.steps / elapsed
    # the gather's cost: end-to-end minus compute, both measured on this run; only where there is a gather to other
    # ranks (world > 1), and never negative (the two passes differ by run-to-run noise where the copy is cheap)
    gather_ms = None
    if world > 1 and gather.get("ms_per_step") is not None:
        gather_ms = max(0.0, gather["ms_per_step"] - elapsed / args.steps * 1e3)
        gather["gather_ms_per_step"] = gather_ms
    result = {
        # BASELINE.json's metric for the headline configuration; other workloads name their own N and batch.
        # "vs HPIPM" is the metric's name: HPIPM cannot be built offline, so max_rel_du_vs_cpu_fp64 below is
        # measured against the fp64 CPU oracle (oracle/cmpc_oracle.c) and HPIPM parity itself is unpinned.
        "metric": ("centroidal QPs/sec (N=10, 13-state/12-input) at batch=4096; max|\u0394u| vs HPIPM"
                   if headline and K == 1 else
                   f"centroidal QPs/sec (N={N}, 13-state/12-input) at batch={B}"
                   f"{'' if K == 1 else f', {K} batches in flight'}; max|du| vs fp64 CPU oracle"),
        "value": value,
        "unit": "QPs/s",
        "n_gpus": n_dev,
        "n_ranks": world,
        "shared_gpu": n_dev < world,
        "devices": dev_ids,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_run": warmup_run,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64" if prec == cm.F64 else "f32",
        "data": "synthetic (Philox4x32-10 counter-based generator, seed 20221125, CentoidMPCTest params)",
        "config": {"workload": f"batch {B} QPs/GPU, N={N}, 13-state/12-input SRBD, "
                               f"{'all-stance (pronk)' if args.all_stance else ('4-contact trot' if args.gait == 0 else 'mixed trot/bound/pronk')}, "
                               f"{'fp64' if prec == cm.F64 else 'fp32'}, full hot path per step",
                   "batch_per_gpu": B, "horizon": N, "parallelism": f"shard{world}"},
        # compute-bound on the vector ALU: the IPM's arithmetic runs on the fp64/fp32 VALU (on gfx950 the VALU issues
        # fp64 at twice the rate of v_mfma_f64_16x16x4); peak = the dtype's vector datasheet peak
        "roofline": roofline,
        **extra,
        "stages_ms": stages,
        "fused_n64": fused,
        "inflight": K,
        "graph": bool(args.graph),
        "path": {k: eng.get_path(getattr(cm, "PATH_" + k)) for k in ("FUSED64", "FUSED128", "DIRECT", "RICCATI", "IPM72")},
        "stage_events": args.stage_events,
        "stage_event_steps": n_prof if timed_events else None,
        "value_end_to_end": value_e2e,
        "value_short_warmup": value_short,
        "cadence": cadence,
        "gather_ms": gather_ms, "gather": gather,
        "build": {"version": cm.lib().cmpc_version().decode(), "lib_md5": lib_md5()},
        "solver": {"success_frac": float(ok.mean()), "mean_iters": float(iters[ok].mean()) if ok.any() else 0.0,
                   "mean_n": float(nvar.mean())},
    }
    if args.sqp_iters > 0:
        si = sqp_si.host()
        result["metric"] = ("centroidal NLP solves/sec by batched SQP (bilinear lever arm"
                            + (", footholds as variables" if args.nlp else "") + "), not the headline metric")
        result["unit"] = "NLPs/s"
        result["solver"]["mean_sqp_iters"] = float(si.mean())
        result["solver"]["mean_iters"] = float(iters[ok].mean()) if ok.any() else 0.0
        result["roofline"] = None

    if rank == 0 and world == 1 and args.cpu_sample > 0 and args.sqp_iters <= 0:
        S = min(args.cpu_sample, B)
        share, share_why = cpu_share()
        threads = args.cpu_threads or share
        hx0, hxr, hft = x0.host()[:S], xref.host()[:S], foot.host()[:S]
        uc, stc, dtc, done = cpu_baseline(N, hx0, hxr, hft, ct[:S], threads)
        ug = u.host()[:S]
        scale = np.maximum(1.0, np.abs(uc).reshape(S, -1).max(axis=1))
        rel = (np.abs(ug - uc).reshape(S, -1).max(axis=1) / scale)
        both = (stc == 0) & (status[:S] == 0)
        result["cpu_baseline"] = {"value": done / dtc, "unit": "QPs/s", "cores": threads, "kind": "port",
                                  "host_cpus": os.cpu_count(), "cpu_share": f"{share} ({share_why})",
                                  "sample": f"first {S} QPs of the same batch x{done // S}, oracle/cmpc_oracle.c "
                                            f"fp64 (same algorithm) built -O3 -march={oracle_fast_build()[1]} "
                                            f"({oracle_fast_build()[0]}), "
                                            f"{threads} pthreads, {dtc:.2f} s wall"}
        result["max_rel_du_vs_cpu_fp64"] = float(rel[both].max()) if both.any() else None
        ur, str_, dtr, doner = cpu_baseline(N, hx0, hxr, hft, ct[:S], threads, riccati=True)
        relr = np.abs(ug - ur).reshape(S, -1).max(axis=1) / np.maximum(1.0, np.abs(ur).reshape(S, -1).max(axis=1))
        bothr = (str_ == 0) & (status[:S] == 0)
        result["cpu_baseline_riccati"] = {
            "value": doner / dtr, "unit": "QPs/s", "cores": threads, "kind": "port",
            "sample": f"first {S} QPs x{doner // S}, oracle_riccati_solve_batch (HPIPM-style: no condensing, Riccati "
                      f"Newton steps over the stages, same IPM), {threads} pthreads, {dtr:.2f} s wall",
            "max_rel_du_vs_gpu": float(relr[bothr].max()) if bothr.any() else None}
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
