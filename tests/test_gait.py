"""Contact schedules from gait templates: GaitSchedule.cpp:78-127 tiling, MotionPhaseDefinition.h
stance decoding. CPU: the built-in templates equal the reference's gait.info (fixture tests/golden/gait_templates.json,
made by tests/golden/make_gait_fixture.py) and the oracle follows the tiling rules; GPU: the device tables are
bit-identical to the oracle's and feed the solver end to end."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gait_templates.json")
MODES = {"FLY": 0, "RH": 1, "LH": 2, "LH_RH": 3, "RF": 4, "RF_RH": 5, "RF_LH": 6, "RF_LH_RH": 7, "LF": 8, "LF_RH": 9,
         "LF_LH": 10, "LF_LH_RH": 11, "LF_RF": 12, "LF_RF_RH": 13, "LF_RF_LH": 14, "STANCE": 15}
# ocs2 leg j -> contact column (CentoidMPCTest.cpp:43-46 order lf, rf, rh, lh)
LEG_MAP = [0, 1, 3, 2]


def fixture():
    with open(GOLD) as f:
        return json.load(f)["gaits"]


def test_builtin_templates_match_reference_gait_info(cmh):
    cm = cmh
    for g in fixture():
        b = cm.gait_builtin(g["name"])
        M = len(g["modeSequence"])
        assert b.n_modes == M, g["name"]
        assert [b.mode[i] for i in range(M)] == [MODES[m] for m in g["modeSequence"]], g["name"]
        assert [b.switching_time[i] for i in range(M + 1)] == g["switchingTimes"], g["name"]
    with pytest.raises(RuntimeError):
        cm.gait_builtin("moonwalk")


def expected(g, t_start, t0, dt, N):
    """Pure-Python restatement: STANCE before t_start, template tiled after (left-closed intervals)."""
    out = np.zeros((N, 4), np.uint8)
    for k in range(N):
        t = t0 + k * dt
        mode = 15
        if not t < t_start:
            M = g.n_modes
            tau = np.fmod(t - t_start, g.switching_time[M] - g.switching_time[0]) + g.switching_time[0]
            i = max(j for j in range(M) if j == 0 or g.switching_time[j] <= tau)
            mode = g.mode[i]
        for j in range(4):
            out[k, LEG_MAP[j]] = (mode >> (3 - j)) & 1
    return out


def test_oracle_gait_semantics(cmh, op):
    cm = cmh
    trot = cm.gait_builtin("trot")
    c = op.gait_contact(trot, 0.0, 0.0, 0.05, 28)
    # LF_RH (lf, rh = columns 0, 2) for [0, 0.35), RF_LH (columns 1, 3) for [0.35, 0.70), repeating
    assert np.array_equal(c[0], [1, 0, 1, 0]) and np.array_equal(c[7], [0, 1, 0, 1]) and np.array_equal(c[14], [1, 0, 1, 0])
    # stance before the template starts
    c = op.gait_contact(trot, 0.2, 0.0, 0.05, 8)
    assert np.all(c[:4] == 1) and np.array_equal(c[4], [1, 0, 1, 0])
    for g in fixture():
        b = cm.gait_builtin(g["name"])
        for ts, t0, dt, N in ((0.0, 0.0, 0.01, 10), (0.13, 0.05, 0.02, 40), (-3.3, 1.7, 0.03, 64)):
            assert np.array_equal(op.gait_contact(b, ts, t0, dt, N), expected(b, ts, t0, dt, N)), g["name"]


@pytest.mark.gpu
def test_device_gait_tables_bit_exact(cm, op):
    gaits = [cm.gait_builtin(g["name"]) for g in fixture()]
    table = cm.GaitTable(gaits)
    rng = np.random.default_rng(9)
    B, N = 513, 20
    ids = rng.integers(0, len(gaits), B).astype(np.int32)
    ts = rng.uniform(-1.0, 1.0, B)
    for t0, dt in ((0.0, 0.01), (0.37, 0.02), (12.5, 0.015)):
        got = table.contact(ids, ts, t0, dt, N)
        for q in range(B):
            assert np.array_equal(got[q], op.gait_contact(gaits[ids[q]], ts[q], t0, dt, N)), (q, ids[q])
    # ids outside the table -> all-swing rows
    got = table.contact(np.array([-1, len(gaits)], np.int32), np.zeros(2), 0.0, 0.01, N)
    assert np.all(got == 0)


@pytest.mark.gpu
def test_schedule_fed_solve_matches_oracle(cm, op):
    """Per-QP gaits from the templates without flight phases -> ragged contact tables -> full hot path."""
    names = ["trot", "standing_trot", "standing_pace", "static_walk", "amble", "dynamic_walk", "stance", "lindyhop"]
    gaits = [cm.gait_builtin(n) for n in names]
    table = cm.GaitTable(gaits)
    N, B = 10, 64
    m, mo = cm.default_model(N), op.default_model(N)
    rng = np.random.default_rng(4)
    ids = rng.integers(0, len(gaits), B).astype(np.int32)
    ts = rng.uniform(0.0, 0.5, B)
    contact = table.contact(ids, ts, 0.0, m.dt, N)
    x0, xref, foot, _ = op.generate(mo, 20221125, B, gait=0)
    eng = cm.Engine(m, precision=0, max_batch=B)
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    ur, xr, sr, itr = op.solve_batch(mo, op.default_settings(), x0, xref, foot, contact, nthreads=8)
    assert np.all(st == sr) and np.all(st == 0)
    nvar = 3 * contact.reshape(B, -1).sum(axis=1)
    assert len(np.unique(nvar)) > 3
    err = max(float(np.max(np.abs(u[q] - ur[q])) / max(1.0, float(np.max(np.abs(ur[q]))))) for q in range(B))
    assert err < 1e-6, err
