"""Regenerates tests/golden/*.npz — run in the dev container: `python tests/golden/make_golden.py`.

Expected outputs come from oracle/np_ref.py, the independent numpy restatement of the reference's CentroidalMPC
model (CentroidalMPC.cpp:41-100 dynamics, :179-201 pyramid, :203-231 cost, :326-335 f^des) — not from the C oracle
and not from the HIP path, so both are checked against it. The reference ships no golden vectors and its solver
(CasADi/IPOPT, HPIPM) is not buildable offline: these fixtures pin the restated algorithm, not the
HPIPM binary. Inputs: CentoidMPCTest.cpp:36-111 (config 1, literal des_state quirk) and the Philox generator
(configs 2/3/5, seed 20221125). Philox4x32-10 known-answer vectors are the published Random123 ones.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import np_ref  # noqa: E402
import oracle_py as op  # noqa: E402  (only for the generator that produces the synthetic inputs)

SEED = 20221125


def case(name, model, x0, xref, foot, contact):
    M = np_ref.model_arrays(model)
    B = x0.shape[0]
    N = model.N
    Hs, gs, us, ns = [], [], [], []
    for q in range(B):
        Hf, gf, _, _ = np_ref.condense_full(M, x0[q], xref[q], foot[q], contact[q])
        Hs.append(Hf)
        gs.append(gf)
        us.append(np_ref.solve(M, x0[q], xref[q], foot[q], contact[q]))
        ns.append(3 * int(contact[q].sum()))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), N=N, x0=x0, xref=xref, foot=foot, contact=contact,
                        H_full=np.array(Hs), g_full=np.array(gs), u=np.array(us), n=np.array(ns))
    print(name, B, "QPs, max|u| =", float(np.abs(np.array(us)).max()))


def main():
    for N in (6, 10):
        x0, xref, foot, contact = np_ref.centoid_test_inputs(N, literal_quirk=True)
        case(f"centoid_mpc_test_N{N}", op.default_model(N), x0[None], xref[None], foot[None], contact[None])
    case("config2_trot_N10", op.default_model(10), *op.generate(op.default_model(10), SEED, 8, gait=0))
    case("config3_trot_N20", op.default_model(20), *op.generate(op.default_model(20), SEED, 3, gait=0))
    case("config5_mixed_N10", op.default_model(10), *op.generate(op.default_model(10), SEED, 8, gait=1))
    kat = np.array([[0, 0, 0, 0, 0, 0, 0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8],
                    [0xffffffff] * 6 + [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd],
                    [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0,
                     0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]], dtype=np.uint32)
    np.savez_compressed(os.path.join(HERE, "philox4x32_10_kat.npz"), kat=kat)


if __name__ == "__main__":
    main()
