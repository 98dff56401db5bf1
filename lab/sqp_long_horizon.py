import sys, os
sys.path[:0] = ['cheeta-mpc_amd/python', 'oracle']
import numpy as np, cheeta_mpc as cm, oracle_py as op
for N in (30, 63):
    B = 8
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, 99, B, gait=0)
    eng = cm.Engine(m, precision=0, max_batch=B)
    u, x, st, qi, si = eng.sqp_solve(x0, xref, foot, contact, sqp_iter_max=5, sqp_tol=1e-7)
    un, fn, xn, stn, qin, sin_ = eng.nlp_solve(x0, xref, foot, contact, sqp_iter_max=5, sqp_tol=1e-7)
    for q in range(B):
        r1 = op.sqp_solve(mo, op.default_settings(), x0[q], xref[q], foot[q], contact[q], 5, 1e-7)
        r2 = op.sqp_solve_feet(mo, op.default_settings(), x0[q], xref[q], foot[q], contact[q], 5, 1e-7)
        n = 3 * int(contact[q].sum())
        e1 = float(np.abs(u[q] - r1[0]).max()) if r1[2] == 0 else 0.0
        e2 = float(np.abs(un[q] - r2[0]).max()) if r2[4] == 0 else 0.0
        print(N, q, n, 'sqp', st[q], r1[2], si[q], r1[4], f'{e1:.1e}', 'nlp', stn[q], r2[4], sin_[q], r2[6], f'{e2:.1e}')
