"""World-size-2 gloo test of the sharded (multi-GPU) path on CPU: every rank takes its contiguous QP-id slice,
generates its inputs from (seed, global id) and solves them (here with the CPU oracle: there is no GPU in this
suite); the gathered shards must equal the single-process batch bit for bit, and the timing reduction is a max."""
import os
import socket
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

WORKER = r"""
import os, sys, time, pickle
sys.path[:0] = [os.path.join(ROOT, 'cheeta-mpc_amd', 'python'), os.path.join(ROOT, 'oracle')]
from cheeta_mpc.shard import Dist, shard_range
import oracle_py as op
d = Dist()
TOTAL = 37
off, cnt = shard_range(TOTAL, d.world, d.rank)
m = op.default_model(10)
x0, xref, foot, contact = op.generate(m, 20221125, cnt, gait=1, offset=off)
u, _, st, it = op.solve_batch(m, op.default_settings(), x0, xref, foot, contact, want_x=False)
d.barrier()
t = d.max(1.0 + d.rank)
parts = d.gather_object((off, cnt, u.tolist(), st.tolist()))
if d.rank == 0:
    with open(OUT, 'wb') as f:
        pickle.dump({'t': t, 'parts': parts}, f)
d.close()
"""


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    from cheeta_mpc.shard import shard_range
    for total in (0, 1, 7, 4096, 262144):
        for world in (1, 2, 3, 8):
            slices = [shard_range(total, world, r) for r in range(world)]
            assert sum(c for _, c in slices) == total
            pos = 0
            for off, c in slices:
                assert off == pos
                pos += c


def test_two_rank_gloo_shards_match_single_process(tmp_path):
    import pickle
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as op
    out = tmp_path / "res.pkl"
    script = tmp_path / "worker.py"
    script.write_text(f"ROOT = {ROOT!r}\nOUT = {str(out)!r}\n" + WORKER)
    port = free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=e))
    for p in procs:
        assert p.wait(timeout=240) == 0
    res = pickle.load(open(out, "rb"))
    assert res["t"] == 2.0
    parts = sorted(res["parts"])
    u = np.concatenate([np.array(p[2]) for p in parts])
    st = np.concatenate([np.array(p[3]) for p in parts])
    m = op.default_model(10)
    x0, xref, foot, contact = op.generate(m, 20221125, 37, gait=1)
    ur, _, sr, _ = op.solve_batch(m, op.default_settings(), x0, xref, foot, contact, want_x=False)
    assert np.array_equal(st, sr)
    assert np.array_equal(u, ur)


GATHER_FAIL_WORKER = r"""
import os, sys, pickle
sys.path[:0] = [os.path.join(ROOT, 'cheeta-mpc_amd', 'python')]
from cheeta_mpc.shard import Dist, ResultGather
import cheeta_mpc as cm
d = Dist()
if d.rank == 0:  # rank 0 cannot export its buffer (stands for a failed hipIpcGetMemHandle / allocation)
    class _Fail:
        def __init__(self, *a, **k):
            raise RuntimeError("export failed on rank 0")
    cm.DeviceArray = _Fail
try:
    ResultGather(d, 1024)
    res = 'no error'
except Exception as e:
    res = type(e).__name__ + ': ' + str(e)
d.barrier()  # the ranks' collectives are still matched after the failure
t = d.max(1.0 + d.rank)
with open(OUT + str(d.rank), 'wb') as f:
    pickle.dump({'res': res, 't': t}, f)
d.close()
"""


def test_result_gather_failure_is_symmetric(tmp_path):
    """A rank that cannot set up the result gather (ResultGather, the xGMI / IPC gather of SURVEY §8e) makes every rank
    raise after the handle exchange instead of leaving the other ranks blocked in a collective: both ranks report the
    failure, and the barrier and the max-reduction that follow still match (no hang)."""
    import pickle
    out = tmp_path / "res"
    script = tmp_path / "worker.py"
    script.write_text(f"ROOT = {ROOT!r}\nOUT = {str(out)!r}\n" + GATHER_FAIL_WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(2)]
    for p in procs:
        assert p.wait(timeout=240) == 0
    r0 = pickle.load(open(str(out) + "0", "rb"))
    r1 = pickle.load(open(str(out) + "1", "rb"))
    assert "export failed on rank 0" in r0["res"]
    assert "rank 0 could not export" in r1["res"]
    assert r0["t"] == r1["t"] == 2.0


STDOUT_WORKER = r"""
import os, sys
sys.path[:0] = [os.path.join(ROOT, 'cheeta-mpc_amd', 'python')]
from cheeta_mpc.shard import Dist
d = Dist()
d.barrier()
if d.rank == 0:
    print('{"value": 1}')
d.close()
"""


def test_rank0_stdout_is_only_the_json_line(tmp_path):
    """bench.py's contract: rank 0 prints one JSON line. gloo's rendezvous message ("[Gloo] Rank r is connected to
    ...") is routed to stderr while the process group forms, so no rank's stdout carries anything else."""
    script = tmp_path / "worker.py"
    script.write_text(f"ROOT = {ROOT!r}\n" + STDOUT_WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True) for r in range(2)]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    assert [p.returncode for p in procs] == [0, 0]
    assert outs[0] == '{"value": 1}\n', outs[0]
    assert outs[1] == "", outs[1]
