"""Independent numpy restatement of the centroidal condensed QP (used to make and check the golden fixtures).

TEST INFRASTRUCTURE ONLY. Written independently of oracle/cmpc_oracle.c (explicit Aqp/Bqp block products and a
difference-operator force-rate term instead of recursions; a stacked-inequality IPM instead of the pyramid-structured
one) so that the two cross-check each other. Follows:
  CentroidalMPC.cpp:85-92   forward-Euler centroidal dynamics, lever arm linearised at p - c^ref,
                            p the stance foot position (:93 pinning; node 0 = current foot, :165-167, :288-291)
  CentroidalMPC.cpp:203-231 cost (CoM-z weight squared, force tracking, force-rate), x2 folded (App. A.3)
  CentroidalMPC.cpp:179-201 friction pyramid + force bounds; swing legs eliminated (App. A.4)
  CentroidalMPC.cpp:326-335 f^des_z = m*9.81/n_stance and the "mpc table invalid" rule
"""
import numpy as np

NX, NU, NL = 13, 12, 4
GRAV = 9.81


def model_arrays(model):
    N = model.N
    w = np.array(model.weights[:45], dtype=np.float64)
    L = model.n_legs
    Wf = np.array([w[9 + 3 * L + j] for j in range(12)])
    Wr = np.array([w[9 + 6 * L + j] for j in range(12)])
    q = np.zeros((N + 1, NX))
    for k in range(N + 1):
        wz = (w[2] / 2.0) * np.exp(-float(k)) + w[2] / 2.0
        q[k] = 2.0 * np.array([w[0], w[1], wz * wz, *w[3:9], *model.theta_weights[:3], 0.0])
    Ib = np.array(model.inertia[:9]).reshape(3, 3)
    return dict(N=N, m=model.mass, dt=model.dt, Wf=Wf, Wr=Wr, q=q, Ibinv=np.linalg.inv(Ib),
                mu=np.array(model.mu[:4]), ub=np.array(model.force_ub[:5]))


def skew(r):
    return np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])


def stance_feet(foot, contact):
    """Foot position behind every stance force, P[k, i] (CentroidalMPC.cpp:93: a stance foot does not move).

    foot[0] is the current foot position (state[9+3i..], :288-291, pinned as foot_pos(:,0) by :165-167), foot[1..N]
    is des_foot_pos. Each maximal stance run of a leg (steps s..e) holds one position over nodes s..e+1: foot[0] for a
    run that starts at step 0, otherwise the mean of des_foot_pos over nodes s..e+1 (the tracking-cost minimiser).
    Restated from run boundaries found with numpy diffs (independent of oracle_stance_point's scans).
    """
    N = contact.shape[0]
    P = np.zeros((N, NL, 3))
    for i in range(NL):
        e = np.concatenate([[0], contact[:, i].astype(np.int64), [0]])
        starts = np.flatnonzero(np.diff(e) == 1)      # first stance step of each run
        ends = np.flatnonzero(np.diff(e) == -1) - 1    # last stance step of each run
        for s0, e0 in zip(starts, ends):
            if s0 == 0:
                pos = foot[0, i]
            else:
                nodes = foot[s0:e0 + 2, i]
                pos = nodes[0] + (nodes - nodes[0]).sum(axis=0) / len(nodes)
            P[s0:e0 + 1, i] = pos
    return P


def dynamics(M, xref, foot, contact):
    N, dt, m = M["N"], M["dt"], M["m"]
    A = np.zeros((N, NX, NX))
    B = np.zeros((N, NX, NU))
    P = stance_feet(foot, contact)
    for k in range(N):
        Ak = np.eye(NX)
        Ak[0:3, 3:6] = dt * np.eye(3)
        Ak[5, 12] = dt
        psi = xref[k, 11]
        Rz = np.array([[np.cos(psi), -np.sin(psi), 0], [np.sin(psi), np.cos(psi), 0], [0, 0, 1]])
        Ak[9:12, 6:9] = dt * (M["Ibinv"] @ Rz.T)
        A[k] = Ak
        for i in range(NL):
            if contact[k, i]:
                B[k, 3:6, 3 * i:3 * i + 3] = dt / m * np.eye(3)
                B[k, 6:9, 3 * i:3 * i + 3] = dt * skew(P[k, i] - xref[k, 0:3])
    return A, B


def condense_full(M, x0, xref, foot, contact):
    """H = Bqp' Qbar Bqp + Rbar, g = Bqp' Qbar (Aqp x0 - Xref) + rbar over all 12N inputs."""
    N = M["N"]
    ns = contact.sum(axis=1)
    if np.any(ns == 0):
        raise ValueError("mpc table invalid")
    A, B = dynamics(M, xref, foot, contact)
    Aqp = np.zeros((N * NX, NX))
    Bqp = np.zeros((N * NX, N * NU))
    for k in range(1, N + 1):           # state x_k
        P = np.eye(NX)
        for j in range(k - 1, -1, -1):  # input u_j, j < k: A_{k-1}...A_{j+1} B_j
            Bqp[(k - 1) * NX:k * NX, j * NU:(j + 1) * NU] = P @ B[j]
            P = P @ A[j]
        Aqp[(k - 1) * NX:k * NX] = P
    Qbar = np.diag(M["q"][1:].reshape(-1))
    Xref = xref[1:].reshape(-1)
    D = np.zeros(((N - 1) * NU, N * NU))
    for k in range(N - 1):
        D[k * NU:(k + 1) * NU, k * NU:(k + 1) * NU] = -np.eye(NU)
        D[k * NU:(k + 1) * NU, (k + 1) * NU:(k + 2) * NU] = np.eye(NU)
    Wf = np.tile(M["Wf"], N)
    Wr = np.tile(M["Wr"], N - 1)
    Rbar = 2.0 * np.diag(Wf) + 2.0 * D.T @ np.diag(Wr) @ D
    fdes = np.zeros((N, NL, 3))
    for k in range(N):
        for i in range(NL):
            if contact[k, i]:
                fdes[k, i, 2] = M["m"] * GRAV / ns[k]
    rbar = -2.0 * Wf * fdes.reshape(-1)
    H = Bqp.T @ Qbar @ Bqp + Rbar
    g = Bqp.T @ Qbar @ (Aqp @ x0 - Xref) + rbar
    return H, g, Aqp, Bqp


def active_index(contact):
    N = contact.shape[0]
    idx = []
    for k in range(N):
        for i in range(NL):
            if contact[k, i]:
                idx += [NU * k + 3 * i + d for d in range(3)]
    return np.array(idx, dtype=np.int64)


def pyramid(mu):
    return np.array([[-1, 0, mu], [1, 0, mu], [0, -1, mu], [0, 1, mu], [0, 0, 1]], dtype=np.float64)


def condense(M, x0, xref, foot, contact):
    H, g, Aqp, Bqp = condense_full(M, x0, xref, foot, contact)
    idx = active_index(contact)
    legs = [i for k in range(contact.shape[0]) for i in range(NL) if contact[k, i]]
    Hr = H[np.ix_(idx, idx)]
    gr = g[idx]
    nt = len(legs)
    C = np.zeros((5 * nt, 3 * nt))
    for t, leg in enumerate(legs):
        C[5 * t:5 * t + 5, 3 * t:3 * t + 3] = pyramid(M["mu"][leg])
    lo = np.zeros(5 * nt)
    hi = np.tile(M["ub"], nt)
    return Hr, gr, C, lo, hi, idx


def ipm_stacked(H, g, C, lo, hi, tol=1e-12, iters=80):
    """min 1/2u'Hu+g'u s.t. Au >= b with A = [C; -C], b = [lo; -hi]; Mehrotra, one step length."""
    n = H.shape[0]
    if n == 0:
        return np.zeros(0), np.zeros(0)
    Am = np.vstack([C, -C])
    b = np.concatenate([lo, -hi])
    m = Am.shape[0]
    u = np.zeros(n)
    s = np.maximum(Am @ u - b, 1.0)
    z = 10.0 / s
    for _ in range(iters):
        rd = H @ u + g - Am.T @ z
        rp = Am @ u - s - b
        mu = s @ z / m
        if np.abs(rd).max() < tol and np.abs(rp).max() < tol and (s * z).max() < tol:
            break
        K = H + Am.T @ np.diag(z / s) @ Am

        def direction(rc):
            rhs = -rd - Am.T @ ((rc + z * rp) / s)
            du = np.linalg.solve(K, rhs)
            ds = Am @ du + rp
            dz = -(rc + z * ds) / s
            return du, ds, dz

        def maxstep(ds, dz):
            a = 1e300
            for v, dv in ((s, ds), (z, dz)):
                neg = dv < 0
                if neg.any():
                    a = min(a, float(np.min(-v[neg] / dv[neg])))
            return a

        du, ds, dz = direction(s * z)
        a = min(1.0, maxstep(ds, dz))
        mua = (s + a * ds) @ (z + a * dz) / m
        sig = (mua / mu) ** 3
        du, ds, dz = direction(s * z + ds * dz - sig * mu)
        a = min(1.0, 0.995 * maxstep(ds, dz))
        u += a * du
        s += a * ds
        z += a * dz
    return u, z


def solve(M, x0, xref, foot, contact):
    """Forces u[N, 4, 3] (zeros for swing) of the condensed QP."""
    Hr, gr, C, lo, hi, idx = condense(M, x0, xref, foot, contact)
    ur, z = ipm_stacked(Hr, gr, C, lo, hi)
    u = np.zeros(M["N"] * NU)
    u[idx] = ur
    return u.reshape(M["N"], NL, 3)


def centoid_test_inputs(N=6, literal_quirk=True):
    """CentoidMPCTest.cpp:36-111 inputs mapped to the 13-state record.

    literal_quirk=True reproduces the release-build layout of the test's under-filled des_state (54 values into a
    63-vector, CentoidMPCTest.cpp:37/:48-65; read by CentroidalMPC.cpp:297-299 as 3x(N+1) column-major blocks): the
    7th c^des column is the first v^des triple and every later block shifts by one column.
    For N > 6 the trot table continues with period 6 and the last desired columns are held.
    """
    state = np.array([0, 0, 0.15, 0.1, 0, 0, 0, 0, 0.1,
                      0.35, 0.052, 0, 0.35, -0.054, 0, -0.37, -0.053, 0, -0.36, 0.054, 0])
    vals = [0.31, 0, 0.16, 0.32, 0, 0.168, 0.33, 0, 0.172, 0.33, 0, 0.18, 0.34, 0, 0.19, 0.348, 0, 0.2,
            0.1, 0, 0, 0.09, 0, 0, 0.08, 0, 0, 0.06, 0, 0, 0.04, 0, 0, 0, 0, 0,
            0, 0, 0.12, 0, 0, 0.14, 0, 0, 0.16, 0, 0, 0.18, 0, 0, 0.2, 0, 0, 0.22]
    des6 = np.zeros(63)
    des6[:54] = vals
    if literal_quirk:
        blocks = [des6[0:21].reshape(7, 3), des6[21:42].reshape(7, 3), des6[42:63].reshape(7, 3)]
    else:
        v = np.array(vals)
        blocks = [np.vstack([v[0:18].reshape(6, 3), v[15:18]]), np.vstack([v[18:36].reshape(6, 3), v[33:36]]),
                  np.vstack([v[36:54].reshape(6, 3), v[51:54]])]
    table6 = np.array([[1, 0, 1, 0]] * 3 + [[0, 1, 0, 1]] * 3, dtype=np.uint8)
    feet6 = np.array([
        [[0.35, 0.052, 0], [0.35, 0.052, 0], [0.35, 0.052, 0], [0.35, 0.052, 0], [0.38, 0.052, 0], [0.39, 0.052, 0],
         [0.42, 0.052, 0]],
        [[0.35, -0.054, 0], [0.37, -0.052, 0], [0.39, -0.052, 0], [0.43, -0.052, 0], [0.43, -0.052, 0],
         [0.43, -0.052, 0], [0.43, -0.052, 0]],
        [[-0.37, -0.052, 0], [-0.37, -0.052, 0], [-0.37, -0.052, 0], [-0.36, -0.052, 0], [-0.34, -0.052, 0],
         [-0.30, -0.052, 0], [-0.28, -0.052, 0]],
        [[-0.36, 0.053, 0], [-0.34, 0.053, 0], [-0.32, 0.053, 0], [-0.31, 0.053, 0], [-0.31, 0.052, 0],
         [-0.31, 0.052, 0], [-0.31, 0.052, 0]]])  # [leg][node][xyz]
    x0 = np.zeros(NX)
    x0[0:9] = state[0:9]
    x0[12] = -GRAV
    xref = np.zeros((N + 1, NX))
    foot = np.zeros((N + 1, NL, 3))
    for k in range(N + 1):
        kk = min(k, 6)
        xref[k, 0:3] = blocks[0][kk]
        xref[k, 3:6] = blocks[1][kk]
        xref[k, 6:9] = blocks[2][kk]
        xref[k, 12] = -GRAV
        foot[k] = feet6[:, kk, :]
    foot[0] = state[9:21].reshape(NL, 3)  # node 0 = cur_foot_pos from the state (CentroidalMPC.cpp:288-291)
    contact = np.zeros((N, NL), dtype=np.uint8)
    for k in range(N):
        contact[k] = table6[k % 6]
    return x0, xref, foot, contact


def ocp_eq_fullspace(N, nx, nu, x0, A, B, b, Q, S, R, q, r, Cc=None, D=None, e=None):
    """HpipmInterface::solve's OCP-QP (HpipmInterface.cpp:166-301) restated in the FULL (x, u) space, independent of
    the device's condensing: decision vector z = [u_0, x_1, u_1, ..., x_N] (x_0 = x0 given), cost
    sum_k 1/2 x'Q x + u'S x + 1/2 u'R u + q'x + r'u, equalities x_{k+1} = A x_k + B u_k + b_k and, when given,
    C_k x_k + D_k u_k + e_k = 0 (the rows the reference passes to HPIPM as lg = ug = -e, :223-264). One dense KKT
    solve (least squares, so consistent redundant rows are fine). Returns (x [N+1][nx], u list, residual of the
    constraint rows)."""
    xo = [None] + [0] * N  # offset of x_k in z (k >= 1)
    uo = [0] * N
    n = 0
    for k in range(N + 1):
        if k >= 1:
            xo[k] = n
            n += nx
        if k < N:
            uo[k] = n
            n += nu[k]
    P = np.zeros((n, n))
    p = np.zeros(n)
    rows, rhs = [], []
    x0 = np.asarray(x0, np.float64)

    def xs(k):
        return slice(xo[k], xo[k] + nx)

    def us(k):
        return slice(uo[k], uo[k] + nu[k])
    for k in range(N + 1):
        m = nu[k] if k < N else 0
        if k >= 1:
            P[xs(k), xs(k)] += Q[k]
            p[xs(k)] += q[k]
        if m:
            P[us(k), us(k)] += R[k]
            p[us(k)] += r[k]
            if k >= 1:
                P[us(k), xs(k)] += S[k]
                P[xs(k), us(k)] += S[k].T
            else:
                p[us(k)] += S[k] @ x0
    for k in range(N):  # dynamics rows: x_{k+1} - A x_k - B u_k = b_k
        row = np.zeros((nx, n))
        row[:, xs(k + 1)] = np.eye(nx)
        rh = np.array(b[k], dtype=np.float64)
        if k >= 1:
            row[:, xs(k)] = -A[k]
        else:
            rh = rh + A[k] @ x0
        if nu[k]:
            row[:, us(k)] = -B[k]
        rows.append(row)
        rhs.append(rh)
    ncon = 0
    if Cc is not None:
        for k in range(N + 1):
            if Cc[k] is None or len(e[k]) == 0:
                continue
            nck = len(e[k])
            row = np.zeros((nck, n))
            rh = -np.asarray(e[k], dtype=np.float64)
            if k >= 1:
                row[:, xs(k)] = Cc[k]
            else:
                rh = rh - Cc[k] @ x0
            if k < N and nu[k]:
                row[:, us(k)] = D[k]
            rows.append(row)
            rhs.append(rh)
            ncon += nck
    Aeq = np.vstack(rows)
    beq = np.concatenate(rhs)
    m_eq = Aeq.shape[0]
    K = np.block([[P, Aeq.T], [Aeq, np.zeros((m_eq, m_eq))]])
    sol = np.linalg.lstsq(K, np.concatenate([-p, beq]), rcond=None)[0]
    z = sol[:n]
    x = np.zeros((N + 1, nx))
    x[0] = x0
    for k in range(1, N + 1):
        x[k] = z[xs(k)]
    u = [z[us(k)] for k in range(N)]
    res = float(np.abs(Aeq @ z - beq).max()) if m_eq else 0.0
    return x, u, res
