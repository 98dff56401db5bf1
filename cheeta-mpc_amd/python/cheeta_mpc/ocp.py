"""Synthetic OCP-QPs of the ocs2_legged_robot SQP subproblem's shape, and record packing for cmpc_ocp_* (cmpc.h).

The reference's only in-repo consumer of HpipmInterface is MultipleShootingSolver on the legged robot
(ocs2_legged_robot/config/mpc/task.info): 24 states (centroidal momentum 6, base pose 6, joint angles 12), 24 inputs
(contact forces 12, joint velocities 12), dt = 0.015 s over a 1.0 s horizon (task.info:33, :102) -> 67 intervals, plus
one event node (no inputs: the jump map, MultipleShootingSolver's PreEvent nodes) per mode switch. Equality
constraints per node (ocs2_legged_robot's LeggedRobotInterface): a stance foot has zero end-effector velocity
(3 rows), a swing foot zero contact force (3 rows) and a normal-velocity reference (1 row). With
projectStateInputEqualityConstraints = true (task.info:40, the robot's setting) ocs2 eliminates them: the QP has no
rows and nu_k = 24 - rows_k inputs (trot: 10, stance: 12, events: 0). With projection off the rows go to HPIPM as
lg = ug rows (HpipmInterface.cpp:223-264).

The matrices are synthetic (random, seeded): A = I + dt Ac, B = dt Bc with entries scaled like a discretised
rigid-body model, diagonal positive state / input weights, force-selection rows for swing feet and random velocity
rows. Data synthetic; shapes and sparsity of the structure as above.
"""
import numpy as np

NX_LEGGED = 24
NU_LEGGED = 24
DT_LEGGED = 0.015


def legged_schedule(N_int=67, period=0.6, dt=DT_LEGGED, stance_time=0.15, t0=0.0):
    """Mode per interval and the event positions of a trot started from full stance: [('stance'|'trotA'|'trotB')],
    with an event node inserted at every mode switch (ocs2's PreEvent nodes). Returns a list of (kind) per node
    k = 0..N-1 where kind in {'stance', 'trotA', 'trotB', 'event'}."""
    kinds = []
    prev = None
    for i in range(N_int):
        t = t0 + i * dt
        if t < stance_time:
            mode = "stance"
        else:
            mode = "trotA" if int((t - stance_time) / (period / 2)) % 2 == 0 else "trotB"
        if prev is not None and mode != prev:
            kinds.append("event")
        kinds.append(mode)
        prev = mode
    return kinds


def _rows_of(kind):
    """(stance feet, swing feet) of a mode: LF, RF, LH, RH; trot pairs {LF, RH} / {RF, LH}."""
    if kind == "stance":
        return [0, 1, 2, 3], []
    if kind == "trotA":
        return [0, 3], [1, 2]
    if kind == "trotB":
        return [1, 2], [0, 3]
    return [], []


def legged_problem(seed=0, projected=True, N_int=67, nx=NX_LEGGED, nu_full=NU_LEGGED, dt=DT_LEGGED,
                   known_solution=False, rows_hold=False, cost="legged", t0=0.0):
    """One synthetic OCP of the legged-robot shape. projected: nu_k = nu_full - rows_k and no rows; else nu_k =
    nu_full (0 at events) and the rows as constraints. known_solution: q, r chosen so that a random (x*, u*)
    rollout is the unconstrained optimum (testHpipmInterface.cpp:112-152); rows_hold: e chosen so the rows hold at
    it (then it is the constrained optimum too). Returns a dict with per-stage lists and x0 (plus xs, us when
    known_solution)."""
    rng = np.random.default_rng(seed)
    kinds = legged_schedule(N_int, dt=dt, t0=t0)
    N = len(kinds)
    nu, nc = [], []
    for kd in kinds:
        st, sw = _rows_of(kd)
        rows = 3 * len(st) + 4 * len(sw)
        if kd == "event":
            nu.append(0)
            nc.append(0)
        elif projected:
            nu.append(nu_full - rows)
            nc.append(0)
        else:
            nu.append(nu_full)
            nc.append(rows)
    nc.append(0)  # terminal node: no rows
    A, B, b, Q, S, R, q, r, Cc, D, e = ([] for _ in range(11))
    for k, kd in enumerate(kinds):
        if kd == "event":  # jump map: identity plus a small reset of the momentum block
            Ak = np.eye(nx)
            Ak[:6, :6] += 0.05 * rng.uniform(-1, 1, (6, 6))
            A.append(Ak)
            B.append(np.zeros((nx, 0)))
            b.append(0.01 * rng.uniform(-1, 1, nx))
        else:
            Ac = np.zeros((nx, nx))
            Ac[6:12, :6] = rng.uniform(-1, 1, (6, 6))           # base pose <- momentum
            Ac[:6, 6:12] = 0.5 * rng.uniform(-1, 1, (6, 6))     # momentum <- pose (gravity torque linearisation)
            Ac += 0.1 * rng.uniform(-1, 1, (nx, nx))
            Bc = np.zeros((nx, nu[k]))
            Bc[:6, :] = rng.uniform(-1, 1, (6, nu[k]))           # momentum <- forces
            Bc[12:, :] = rng.uniform(-1, 1, (nx - 12, nu[k]))    # joints <- joint velocities
            A.append(np.eye(nx) + dt * Ac)
            B.append(dt * Bc)
            b.append(dt * rng.uniform(-1, 1, nx))
    for k in range(N + 1):
        m = nu[k] if k < N else 0
        if cost == "random":
            Mx = rng.uniform(-1, 1, (nx + m, nx + m))
            Hk = Mx @ Mx.T + (nx + m) * np.eye(nx + m)
            Qk, Sk, Rk = Hk[:nx, :nx], Hk[nx:, :nx], Hk[nx:, nx:]
        else:
            w = rng.uniform(1.0, 10.0, nx) * (dt if k < N else 5.0)
            Qk = np.diag(w)
            Rk = np.diag(rng.uniform(0.01, 0.1, m)) * dt if m else np.zeros((0, 0))
            Sk = 0.01 * dt * rng.uniform(-1, 1, (m, nx)) if m else np.zeros((0, nx))
        Q.append(Qk)
        R.append(Rk)
        S.append(Sk)
        q.append(rng.uniform(-1, 1, nx) * dt)
        r.append(rng.uniform(-1, 1, m) * dt)
        g = nc[k]
        if g:
            st, sw = _rows_of(kinds[k])
            Ck = np.zeros((g, nx))
            Dk = np.zeros((g, m))
            row = 0
            for f in st:  # zero foot velocity: J_q qdot (joint-velocity inputs) + base terms (state)
                Ck[row:row + 3, 6:12] = rng.uniform(-1, 1, (3, 6))
                Dk[row:row + 3, 12 + 3 * f:12 + 3 * f + 3] = rng.uniform(0.5, 1.5, (3, 3)) * np.eye(3) + \
                    0.1 * rng.uniform(-1, 1, (3, 3))
                row += 3
            for f in sw:  # zero force (3) and a normal-velocity row (1)
                Dk[row:row + 3, 3 * f:3 * f + 3] = np.eye(3)
                row += 3
                Ck[row, 6:12] = rng.uniform(-1, 1, 6)
                Dk[row, 12 + 3 * f + 2] = 1.0
                row += 1
            Cc.append(Ck)
            D.append(Dk)
            e.append(0.1 * rng.uniform(-1, 1, g))
        else:
            Cc.append(np.zeros((0, nx)))
            D.append(np.zeros((0, m)))
            e.append(np.zeros(0))
    x0 = 0.1 * rng.uniform(-1, 1, nx)
    p = dict(N=N, nx=nx, nu=nu, nc=nc if not projected else None, kinds=kinds, x0=x0, A=A, B=B, b=b, Q=Q, S=S, R=R,
             q=q, r=r, Cc=Cc, D=D, e=e)
    if known_solution:
        xs = [x0]
        us = []
        for k in range(N):
            us.append(rng.uniform(-1, 1, nu[k]))
            xs.append(b[k] + A[k] @ xs[k] + B[k] @ us[k])
            q[k] = -(Q[k] @ xs[k] + S[k].T @ us[k])
            r[k] = -(R[k] @ us[k] + S[k] @ xs[k])
        q[N] = -Q[N] @ xs[N]
        p["xs"] = np.array(xs)
        p["us"] = us
        if rows_hold:
            for k in range(N + 1):
                if p["nc"] is not None and p["nc"][k]:
                    Du = D[k] @ us[k] if k < N else 0.0
                    e[k] = -(Cc[k] @ xs[k] + Du)
    return p


def pack(p):
    """(rec, crec) column-major records of cmpc_ocp_record_size / cmpc_ocp_constraint_record_size."""
    N, nx, nu = p["N"], p["nx"], p["nu"]
    parts = []
    for k in range(N):
        parts += [np.asarray(p["A"][k]).reshape(nx, nx).flatten(order="F"),
                  np.asarray(p["B"][k]).reshape(nx, nu[k]).flatten(order="F"), np.asarray(p["b"][k]).reshape(nx)]
    for k in range(N + 1):
        m = nu[k] if k < N else 0
        parts += [np.asarray(p["Q"][k]).reshape(nx, nx).flatten(order="F"),
                  np.asarray(p["S"][k]).reshape(m, nx).flatten(order="F"),
                  np.asarray(p["R"][k]).reshape(m, m).flatten(order="F"),
                  np.asarray(p["q"][k]).reshape(nx), np.asarray(p["r"][k]).reshape(m)]
    rec = np.concatenate(parts).astype(np.float64)
    crec = None
    nc = p.get("nc")
    if nc is not None:
        cp = []
        for k in range(N + 1):
            m = nu[k] if k < N else 0
            if nc[k] == 0:
                continue
            cp += [np.asarray(p["Cc"][k]).reshape(nc[k], nx).flatten(order="F"),
                   np.asarray(p["D"][k]).reshape(nc[k], m).flatten(order="F"), np.asarray(p["e"][k]).reshape(nc[k])]
        crec = np.concatenate(cp).astype(np.float64) if cp else np.zeros(0)
    return rec, crec
