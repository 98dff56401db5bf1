#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X batched centroidal-MPC QP engine.

Metric (BASELINE.json): centroidal QPs/sec (N=10, 13-state/12-input) at batch=4096, max|du| vs the fp64 reference.
One "step" = one cmpc_solve_batch over a batch of synthetic QPs already resident in HBM: SRBD linearisation +
condensing + pyramid stacking + batched IPM + scatter/rollout (the whole hot path, nothing skipped).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N      (one process per GPU)

Multi-GPU: the QP batch shards with no data-path collective (weak scaling, B per GPU, QP ids offset by rank so every
QP's inputs are the same whatever the sharding); gloo is used only for the start/stop barriers and the max-over-ranks
time. Rank 0 prints one JSON line.
"""
import argparse
import json
import os
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


def cpu_baseline(model_n, x0, xref, foot, contact, threads, min_cpu_s=10.0, max_wall_s=5.0, riccati=False):
    """The CPU oracle (same algorithm, fp64; the -O3 liboracle_fast.so build) on a bounded sample of the same batch,
    repeated until it has done about min_cpu_s of thread-time (capped at max_wall_s wall): QPs/s = QPs solved / wall
    time. riccati=True times the HPIPM-style restatement instead (no condensing; Riccati Newton steps over the stages,
    same iterates)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as op  # test infrastructure: the CPU restatement, timed as the baseline
    op.select_build("liboracle_fast.so")
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
    """HBM bytes per launch of the kernels whose name contains `prefix`, from the committed rocprofv3 --pmc summary
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
    tot = sum(v["hbm_bytes"] for k, v in doc["kernels"].items() if prefix in k)
    return (tot if tot > 0 else None), os.path.basename(path)


def pmc_sq(wkey, prefix):
    """Per-dispatch SQ counters of the kernel whose name contains `prefix`, from the committed rocprofv3 --pmc summary
    of this workload (profiles/pmc_sq_<workload key>.json, cheeta-mpc_amd/tools/pmc_summary.py), only when it was
    taken on this exact build of libcmpc.so (md5)."""
    path = os.path.join(ROOT, "profiles", f"pmc_sq_{wkey}.json")
    if not os.path.exists(path):
        return None, "no SQ PMC summary for this workload"
    with open(path) as f:
        doc = json.load(f)
    if doc.get("lib_md5") != lib_md5():
        return None, f"SQ PMC summary {os.path.basename(path)} was taken on another build of libcmpc.so"
    for k, v in doc["kernels"].items():
        if prefix in k:
            return v["counters"], os.path.basename(path)
    return None, f"{prefix} not in {os.path.basename(path)}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="QPs per GPU per step")
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--precision", choices=["f64", "f32"], default="f64")
    ap.add_argument("--gait", type=int, default=0, help="0 trot (configs 2-4), 1 mixed trot/bound/pronk (config 5)")
    ap.add_argument("--all-stance", action="store_true",
                    help="every leg in stance at every step (pronk): n = 12 N, the largest condensed size class")
    ap.add_argument("--sqp-iters", type=int, default=0,
                    help="> 0: one step = the batched SQP on the bilinear NLP (cmpc_sqp_solve_batch), this many "
                         "SQP iterations at most; not the headline metric")
    ap.add_argument("--inflight", type=int, default=1,
                    help="independent batches in flight: step i runs on context / stream i %% K (a serving pattern; "
                         "each step is still one full batch through the whole hot path). Default 1: the headline")
    ap.add_argument("--stage-events", choices=["timed", "after"], default="timed",
                    help="timed: HIP events around every stage of every timed step (the roofline's kernel times come "
                         "from the timed region itself); after: the timed steps run without events and the stage times "
                         "come from as many profiled steps run right after them")
    ap.add_argument("--cpu-sample", type=int, default=4096, help="QPs in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host's CPU share (cpu_share())")
    ap.add_argument("--traffic-json", default="",
                    help="PMC summary giving roofline.traffic (default: profiles/traffic_<workload key>.json)")
    args = ap.parse_args()

    import cheeta_mpc as cm
    from cheeta_mpc.shard import Dist
    dist = Dist()  # gloo barriers + max-over-ranks only; no collective on the data path
    world, rank = dist.world, dist.rank
    ndev = cm.device_count()
    if ndev <= 0:
        raise RuntimeError("bench.py: no HIP device visible")
    # one GPU per rank; the modulo covers launchers that expose only the rank's own GPU (HIP_VISIBLE_DEVICES)
    cm._hchk(cm.hip().hipSetDevice(dist.local_rank % ndev), "hipSetDevice")
    barrier, max_over_ranks = dist.barrier, dist.max

    B, N = args.batch, args.horizon
    prec = cm.F64 if args.precision == "f64" else cm.F32
    model = cm.default_model(N)
    if prec == cm.F64:
        settings = cm.default_settings()
    else:
        settings = cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4)
    K = max(1, args.inflight)
    engs = [cm.Engine(model, settings, precision=prec, max_batch=B) for _ in range(K)]
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

    def step(i):
        e, (uo, so, io), sh = engs[i % K], outs[i % K], streams[i % K]
        if args.sqp_iters > 0:
            cm.lib().cmpc_sqp_solve_batch(e.ctx, B, x0.ptr, xref.ptr, foot.ptr, contact.ptr, args.sqp_iters, 1e-6,
                                          uo.ptr, None, so.ptr, sqp_qi.ptr, sqp_si.ptr, sh)
        else:
            e.solve_device(B, x0, xref, foot, contact, uo, None, so, io, sh)

    for i in range(args.warmup):
        step(i)
    H.hipDeviceSynchronize()

    timed_events = args.stage_events == "timed"
    if timed_events:
        cm.lib().cmpc_profile_begin(eng.ctx, (args.steps + K - 1) // K)
    barrier()
    H.hipDeviceSynchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
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
            step(i)
        H.hipDeviceSynchronize()
    ms = [C.c_double(0), C.c_double(0), C.c_double(0)]
    ncalls = C.c_int(0)
    cm.lib().cmpc_profile_end(eng.ctx, *[C.byref(m) for m in ms], C.byref(ncalls))
    # stage 1 / 2 / 3 (cmpc.h): condensing / IPM / expand, or on the fused path fused n<=64 / bigger classes / expand
    ms_cond, ms_ipm, ms_exp = (m.value / max(ncalls.value, 1) for m in ms)

    # result gather beside the timed region ("xGMI only for result gather"): every rank writes its U
    # shard into rank 0's buffer (IPC-mapped device-to-device copy; no collective). A failure is reported, not fatal.
    gather = {"what": "U of every rank into rank 0's GPU (cmpc_ipc_open + cmpc_gather_shard), after the timed steps",
              "bytes": world * B * N * 12 * 8, "ms": 0.0 if world == 1 else None}
    if world > 1:
        # ResultGather's constructor and gather() reach every collective on every rank and raise on all ranks
        # together, so the collectives below stay matched whatever fails
        try:
            from cheeta_mpc.shard import ResultGather
            row = N * 12 * 8
            rg = ResultGather(dist, world * B * row)
            barrier()
            tg = time.perf_counter()
            try:
                rg.gather(u.ptr, rank * B * row, B * row, stream)
                gather["ms"] = max_over_ranks(time.perf_counter() - tg) * 1e3
            finally:
                rg.close()
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            gather["error"] = repr(e)[:200]

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
        r_big = roof("bigger classes (k_srbd_condense + k_ipm128x n<=128 / k_ipm_tiled n<=256)", f_big, ms_ipm,
                     "valu", "k_ipm1", "IPM + condensing FLOPs of the n>64 QPs")
        roofline, other = (r_small, r_big) if ms_cond >= ms_ipm else (r_big, r_small)
        stages = {"solve64_fused": ms_cond, "bigger_classes": ms_ipm, "expand": ms_exp}
        f_all = f_small + f_big
        extra = {"roofline_other_stage": other,
                 "roofline_solve": roof("whole solve (all classes, condensing + IPM)", f_all, ms_cond + ms_ipm,
                                        "valu", "cmpc::k_", "IPM + condensing FLOPs of every QP")}
        # the condensing's H = Bqp' Q Bqp contraction inside k_solve64 runs on the matrix cores: its MFMA rate and
        # busy fraction from the committed SQ counters of this build (executed MFMA FLOPs = MOPS x 512)
        c, src = pmc_sq(wkey, "k_solve64")
        mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F64" if prec == cm.F64 else "SQ_INSTS_VALU_MFMA_MOPS_F32") if c else None
        if mops is not None and ms_cond > 0:
            mfl = 512.0 * mops
            cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0  # GRBM_GUI_ACTIVE sums the 8 XCDs
            extra["mfma_condensing"] = {
                "kernel": "k_solve64 condensing phase (H = Bqp' Q Bqp on v_mfma_%s_16x16x4), rate over the fused "
                          "kernel's duration" % ("f64" if prec == cm.F64 else "f32"),
                "mfma_flops_per_launch": mfl, "achieved": mfl / (ms_cond * 1e-3) / 1e12, "peak": peak / 1e12,
                "unit": "TFLOP/s", "frac": mfl / (ms_cond * 1e-3) / peak,
                "mfma_busy_frac": (c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0)
                                   if cyc > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in c else None),
                "source": src}
        else:
            extra["mfma_condensing"] = {"kernel": "k_solve64 condensing phase", "achieved": None, "source": src}
    else:
        roofline = roof("IPM stage (k_ipm64 n<=64, k_ipm128x n<=128, k_ipm_tiled<16> n<=256)", float(fl_ipm.sum()),
                        ms_ipm, "valu", "k_ipm", "IPM FLOPs")
        stages = {"condense": ms_cond, "ipm": ms_ipm, "expand": ms_exp}
        # the condensing stage's Bqp' Q Bqp contraction runs on MFMA (v_mfma_f64_16x16x4 / f32_16x16x4)
        extra = {"roofline_condense": roof("condensing stage (k_condense64 / k_srbd_condense)", float(fl_cond.sum()),
                                           ms_cond, "mfma", "condense", "condensing FLOPs")}

    value = world * B * args.steps / elapsed
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
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
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
        "stage_events": args.stage_events,
        "gather_ms": gather["ms"], "gather": gather,
        "solver": {"success_frac": float(ok.mean()), "mean_iters": float(iters[ok].mean()) if ok.any() else 0.0,
                   "mean_n": float(nvar.mean())},
    }
    if args.sqp_iters > 0:
        si = sqp_si.host()
        result["metric"] = "centroidal NLP solves/sec by batched SQP (bilinear lever arm), not the headline metric"
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
                                            f"fp64 (same algorithm) built -O3 -march=x86-64-v3 (liboracle_fast.so), "
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
