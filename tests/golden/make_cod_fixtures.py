#!/usr/bin/env python3
"""Generate tests/golden/cod_fixtures.json: least-squares systems solved by the REFERENCE's own vendored Eigen
(oracle/_ref/cod_ref, built by `make -C oracle ref` from /root/reference/src/Eigen) exactly as renderROMIS solves
them (A.completeOrthogonalDecomposition().solve(b), src/rendering/render_utils.h:52).

Cases: random dense, sums of outer products like R-OMIS's technique matrices (full rank, rank-deficient, tiny
scale), the zero matrix, and technique matrices / contribution vectors taken from an oracle R-OMIS run.  Run in
the build container only (the GPU box has no /root/reference):  python tests/golden/make_cod_fixtures.py
"""
import json
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def cases():
    rng = np.random.default_rng(20261016)
    out = []
    for t in range(160):
        n = int(rng.integers(1, 9))
        kind = t % 5
        if kind == 0:
            A = rng.standard_normal((n, n)).astype(np.float32)
        elif kind == 1:
            V = rng.random((3 * n, n)).astype(np.float32)
            A = (V.T @ V).astype(np.float32)
        elif kind == 2:
            r = int(rng.integers(0, n + 1))
            V = rng.random((r, n)).astype(np.float32)
            A = (V.T @ V).astype(np.float32)
        elif kind == 3:
            A = np.zeros((n, n), np.float32)
            if t % 2:
                A[0, 0] = np.float32(rng.random())
        else:
            V = (rng.random((2, n)) * 1e-3).astype(np.float32)
            A = (V.T @ V).astype(np.float32)
        out.append((A, rng.standard_normal(n).astype(np.float32), kind))
    # technique matrices of an oracle R-OMIS run (nightclub, 24x16, k = 5, N = 2, 5 iterations)
    from oracle import pyoracle
    from romis_amd import _abi, scene
    W, H = 24, 16
    sc = scene.bench_scene("nightclub_128pt")
    cam = scene.camera_for("nightclub_128pt", W, H)
    osc = pyoracle.OracleScene(sc)
    f = _abi.default_features(ray_trace_mode=_abi.MODE_ROMIS, num_samples_in_reservoir=2)
    n_t, p_mat = pyoracle.gbuffer(osc, cam, W, H)
    seed = _abi.RESTIR_DEFAULT_SEED
    L = pyoracle.lib()
    nbr = pyoracle.neighbours(osc, f, L.or_rng_key(seed, 0, 4, 0), L.or_rng_key(seed, 0, 4, 1), W, H, n_t, p_mat)
    acc = np.zeros((pyoracle.mis_acc_rows(f), W * H), np.float32)
    origin = np.asarray(list(pyoracle.camera_frame(cam).origin), np.float32)
    for it in range(5):
        a, b, d = pyoracle.ris(osc, f, L.or_rng_key(seed, 0, 1, it), origin, W, H, n_t, p_mat)
        pyoracle.romis_accumulate(osc, f, origin, W, H, n_t, p_mat, nbr, a, b, d, it, acc)
    T = 6
    for p in range(0, W * H, 9):
        A = acc[:T * T, p].reshape(T, T).T.copy()          # column-major rows -> A[i, j]
        for c in range(3):
            bv = acc[T * T + c * T:T * T + (c + 1) * T, p].copy()
            out.append((A.astype(np.float32), bv.astype(np.float32), 5))
    return out


def main():
    ref = os.path.join(ROOT, "oracle", "_ref", "cod_ref")
    if not os.path.exists(ref):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
    cs = cases()
    buf = b"".join(struct.pack("<I", A.shape[0]) + np.ascontiguousarray(A.T).tobytes() + b.tobytes() for A, b, _ in cs)
    res = subprocess.run([ref], input=buf, capture_output=True, check=True).stdout
    off = 0
    recs = []
    for A, b, kind in cs:
        n = A.shape[0]
        rank = struct.unpack_from("<I", res, off)[0]
        off += 4
        x = np.frombuffer(res, np.float32, n, off)
        off += 4 * n
        recs.append({"kind": kind, "n": n, "A": A.view(np.uint32).ravel().tolist(), "b": b.view(np.uint32).tolist(),
                     "x": x.view(np.uint32).tolist(), "rank": rank})
    doc = {"generator": "tests/golden/make_cod_fixtures.py",
           "reference": "oracle/_ref/cod_ref: Eigen (vendored at /root/reference/src/Eigen) "
                        "CompleteOrthogonalDecomposition<MatrixXf>::solve, g++ -O2 x86-64 (SSE vectorised)",
           "encoding": "float32 bit patterns; A row-major [n][n]",
           "kinds": {"0": "dense normal", "1": "V^T V full rank", "2": "V^T V rank r <= n", "3": "zero / one entry",
                     "4": "tiny V^T V", "5": "oracle R-OMIS technique matrix + contribution vector"},
           "cases": recs}
    with open(os.path.join(ROOT, "tests", "golden", "cod_fixtures.json"), "w") as fh:
        json.dump(doc, fh, separators=(",", ":"))
    print(len(recs), "cases")


if __name__ == "__main__":
    main()
