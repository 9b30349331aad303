"""Shared helpers for the parity tests."""
import numpy as np

# fp32 parity bound (north_star: "fp32 embeddings within 1e-5 relative"): relative to the
# magnitude of the computation, i.e. |got - ref_f64| <= RTOL * Σ|terms| element-wise. A plain
# |ref| denominator is meaningless for outputs that cancel to ~0.
RTOL = 1e-5


def assert_close(got, ref, mag, rtol=RTOL, what=""):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    mag = np.asarray(mag, dtype=np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = np.abs(got - ref)
    bound = rtol * mag + 1e-30
    bad = err > bound
    if bad.any():
        i = np.argwhere(bad)[0]
        raise AssertionError(
            f"{what}: {bad.sum()} / {bad.size} elements out of tolerance; first at {tuple(i)}: "
            f"got {got[tuple(i)]!r} ref {ref[tuple(i)]!r} mag {mag[tuple(i)]!r} "
            f"(max rel err {np.max(err / (mag + 1e-30)):.3e})")


def random_coo(rng, n_rows, n_cols, nnz, sort=True, dup=False):
    r = rng.integers(0, n_rows, size=nnz)
    c = rng.integers(0, n_cols, size=nnz)
    if not dup:
        key = np.unique(r * n_cols + c)
        r, c = key // n_cols, key % n_cols
        if not sort:
            p = rng.permutation(len(r))
            r, c = r[p], c[p]
    elif sort:
        p = np.argsort(r, kind="stable")
        r, c = r[p], c[p]
    return r.astype(np.int64), c.astype(np.int64)
