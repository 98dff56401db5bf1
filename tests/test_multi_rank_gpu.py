"""Config 4 (BASELINE.json: batch 262144 QPs sharded across GPUs, xGMI gather only) on the device.

* The full 262144-QP batch on one GPU (the whole of config 4's work, ~9 GB of workspace at ld = 64), checked through
  size-independent properties on every QP plus a seeded 64-QP sample against the CPU oracle.
* A world-size-2 run of the HIP path: each rank (own process) solves its contiguous shard with cmpc_solve_batch and
  writes it into rank 0's buffer through cheeta_mpc.shard.ResultGather (dmabuf IPC mapping + one device-to-device
  copy per rank, the xGMI peer write of the 8-GPU node); rank 0 checks the gathered result bit for bit against the
  single-process solve of the whole batch. On a one-GPU box both ranks share the device, which exercises the same
  code path (IPC export/open, the offset copy, the barrier ordering).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from test_full_size import _check_properties, _run, _sample_vs_oracle

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SEED4 = 20221126  # config 4 seed


@pytest.mark.gpu
def test_config4_full_batch_one_gpu(cm, op):
    N, B = 10, 262144
    inputs, u, st, it = _run(cm, N, B, 0, 0, seed=SEED4)
    _check_properties(u, st, it, inputs[3])
    idx = np.sort(np.random.default_rng(4).choice(B, 64, replace=False))
    _sample_vs_oracle(op, N, inputs, u, st, it, idx, 1e-8, True)


WORKER = r"""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.path.join(ROOT, 'cheeta-mpc_amd', 'python'))
import cheeta_mpc as cm
from cheeta_mpc.shard import Dist, ResultGather, shard_range
d = Dist()
ndev = cm.device_count()
cm._hchk(cm.hip().hipSetDevice(d.local_rank % ndev), 'hipSetDevice')
N = 10
off, cnt = shard_range(TOTAL, d.world, d.rank)
m = cm.default_model(N)
eng = cm.Engine(m, precision=0, max_batch=cnt)
x0, xref, foot, contact = cm.generate_device(m, SEED, cnt, gait=1, offset=off)
u = cm.DeviceArray((cnt, N, 4, 3), np.float64)
st = cm.DeviceArray((cnt,), np.int32)
it = cm.DeviceArray((cnt,), np.int32)
stream = C.c_void_p()
cm.hip().hipStreamCreate(C.byref(stream))
eng.solve_device(cnt, x0, xref, foot, contact, u, None, st, it, stream)
row = N * 4 * 3 * 8
g = ResultGather(d, TOTAL * row)
gs = ResultGather(d, TOTAL * 4)
g.gather(u.ptr, off * row, cnt * row, stream)
gs.gather(st.ptr, off * 4, cnt * 4, stream)
if d.rank == 0:
    np.save(OUT + '_u.npy', g.host(np.float64, (TOTAL, N, 4, 3)))
    np.save(OUT + '_st.npy', gs.host(np.int32, (TOTAL,)))
d.barrier()
g.close()
gs.close()
d.close()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_two_rank_hip_shards_gather_bit_exact(cm, tmp_path):
    total = 2 * 2048 + 37  # ragged: the ranks get 2067 and 2066 QPs
    out = str(tmp_path / "gath")
    script = tmp_path / "worker.py"
    script.write_text(f"ROOT = {ROOT!r}\nOUT = {out!r}\nTOTAL = {total}\nSEED = 20221125\n" + WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(2)]
    try:
        rcs = [p.wait(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0]
    ug, sg = np.load(out + "_u.npy"), np.load(out + "_st.npy")
    N = 10
    m = cm.default_model(N)
    eng = cm.Engine(m, precision=0, max_batch=total)
    x0, xref, foot, contact = cm.generate_device(m, 20221125, total, gait=1)
    u = cm.DeviceArray((total, N, 4, 3), np.float64)
    st = cm.DeviceArray((total,), np.int32)
    it = cm.DeviceArray((total,), np.int32)
    eng.solve_device(total, x0, xref, foot, contact, u, None, st, it)
    assert np.array_equal(sg, st.host())
    assert np.array_equal(ug, u.host())
