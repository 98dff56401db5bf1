"""fp32 contexts on the foothold NLP: statuses / iterations of the NLP, the frozen SQP and the foothold QPs alone."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", p) for p in ("cheeta-mpc_amd/python", "oracle", "tests")]
import numpy as np
import cheeta_mpc as cm
import oracle_py as op
from test_feet import later_runs

SEED = 20221125
for N, gait in ((10, 1), (10, 2), (20, 1)):
    B = 16
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=gait)
    for prec in (0, 1):
        eng = cm.Engine(m, precision=prec, max_batch=B)
        u, feet, x, st, qi, si = eng.nlp_solve(x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7)
        us, xs, sts, qis, sis = eng.sqp_solve(x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7)
        print(N, gait, prec, "nlp st", st.tolist(), "qi", qi.tolist(), "si", si.tolist())
        print(N, gait, prec, "sqp st", sts.tolist(), "qi", qis.tolist())
    # the first foothold QP of each problem alone, fp32 vs fp64
    s = op.default_settings()
    Hs, gs, ns, mus, los, his = [], [], [], [], [], []
    ld = cm.Engine(m, precision=1, max_batch=B).ld
    for q in range(B):
        u0 = op.solve_batch(mo, s, x0[q:q+1], xref[q:q+1], foot[q:q+1], contact[q:q+1])[0][0]
        D0 = op.feet_init(mo, foot[q], contact[q])
        lin = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], u0, D0)[2]
        n, H, g, mu, lo, hi, mp, stc = op.condense_feet(mo, x0[q], xref[q], foot[q], contact[q], lin, u0, D0, ld=ld)
        Hs.append(H); gs.append(g); ns.append(n); mus.append(mu); los.append(lo); his.append(hi)
        r = op.qp_ipm(n, H, g, mu, lo, hi, s)
        print("oracle fp64 QP", q, "n", n, "status/iters", r[3], r[4])
    for prec in (0, 1):
        eng = cm.Engine(m, precision=prec, max_batch=B)
        res = eng.qp_solve(np.array(Hs), np.array(gs), np.array(ns, np.int32), np.array(mus), np.array(los), np.array(his))
        print("device QP prec", prec, "status", res[1].tolist(), "iters", res[2].tolist())
