"""The incidence-object layer of the C ABI (hgd_incidence_*, hgd_conv2hop_*, hgd_comm_*;
include/hgd.h "Incidence objects"), called through ctypes exactly as a native host would:

* the object's derived structure (CSC, CSC→CSR permutation, scales) is bit-identical to the
  Python Incidence's (same primitives), and its conv2hop forward/backward is bit-identical to
  functional.two_hop and within the 1e-5 magnitude bound of the float64 oracle
  (HGNN_HD4.py:455-462, EquivSetConv2.py:88-93, data/graph.py:28-42);
* drop-edge children match Incidence.drop / the oracle's SpAdjDropEdge (HCCF.py:213-226),
  including the 1/keep values of a binary parent;
* from_dense matches torch.nonzero (EquivSetGNN2.py:105-133);
* malformed structures are rejected; a one-rank RCCL communicator leaves results unchanged.
"""
import ctypes
import zlib

import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from tests._util import assert_close, random_coo

pytestmark = pytest.mark.gpu

K = {None: 0, "mean": 1, "sym": 2, "wmean": 3, "wsym": 4}
EPI = {None: 0, "leaky_relu": 1, "relu": 2}


def _lib():
    from hypergraph_diffusion_for_recommendation_amd import _native
    return _native, _native.load()


def _st(dev):
    return torch.cuda.current_stream(dev).cuda_stream


class Obj:
    """Owns one hgd_incidence* (destroyed with the Python object)."""

    def __init__(self, handle):
        self.h = handle

    def __del__(self):
        nat, lib = _lib()
        if self.h:
            lib.hgd_incidence_destroy(self.h)
            self.h = None

    def view(self):
        nat, lib = _lib()
        v = nat.IncidenceView()
        nat.check(lib.hgd_incidence_get_view(self.h, ctypes.byref(v)), "get_view")
        return v

    def scale(self, side, kind):
        nat, lib = _lib()
        p = ctypes.c_void_p()
        nat.check(lib.hgd_incidence_scale(self.h, side, K[kind], ctypes.byref(p)), "scale")
        return p.value


def _create(rowptr, col, val, n_rows, n_cols, dev):
    nat, lib = _lib()
    h = ctypes.c_void_p()
    nat.check(lib.hgd_incidence_create(rowptr.data_ptr(), col.data_ptr() if col.numel() else None,
                                       nat.ptr(val), n_rows, n_cols, col.numel(),
                                       ctypes.byref(h), _st(dev)), "hgd_incidence_create")
    return Obj(h.value)


def _dev_array(ptr, n, dtype, dev):
    """Copies n elements at a device pointer into a new tensor (via a raw memcpy)."""
    out = torch.empty(n, dtype=dtype, device=dev)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        torch.cuda.synchronize(dev)
        assert hip.hipMemcpy(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ptr),
                             ctypes.c_size_t(n * out.element_size()), 3) == 0
    return out


def _csr_of(rows, cols, n_rows, dev, shuffle_within_rows=False, rng=None):
    order = np.lexsort((cols, rows))
    r, c = rows[order], cols[order]
    if shuffle_within_rows:
        # columns need not be sorted inside a row
        key = rng.random(len(r))
        order = np.lexsort((key, r))
        r, c = r[order], c[order]
    rowptr = np.zeros(n_rows + 1, np.int64)
    np.add.at(rowptr, r + 1, 1)
    rowptr = np.cumsum(rowptr)
    return (torch.from_numpy(rowptr).to(dev), torch.from_numpy(c.astype(np.int32)).to(dev), r, c)


def _conv(obj, P, Q, R, X, epi, slope, dev, comm=None):
    nat, lib = _lib()
    n_rows, n_cols = obj.view().n_rows, obj.view().n_cols
    d = X.shape[1]
    ws = torch.empty(max(1, lib.hgd_conv2hop_workspace_size(obj.h, d, EPI[epi])),
                     dtype=torch.uint8, device=dev)
    Y = torch.empty(n_rows, d, device=dev)
    M = torch.empty(n_cols, d, device=dev)
    pre = torch.empty(n_rows, d, device=dev) if (epi and slope < 0) else None
    nat.check(lib.hgd_conv2hop_forward(obj.h, K[P], K[Q], K[R], X.data_ptr(), X.stride(0), d,
                                       Y.data_ptr(), d, EPI[epi], float(slope), M.data_ptr(),
                                       nat.ptr(pre), comm, ws.data_ptr(), ws.numel(), _st(dev)),
              "hgd_conv2hop_forward")
    return Y, M, pre, ws


def _conv_bwd(obj, P, Q, R, dY, ref, epi, slope, dev, ws, comm=None):
    nat, lib = _lib()
    n_rows, d = dY.shape
    dX = torch.empty(n_rows, d, device=dev)
    nat.check(lib.hgd_conv2hop_backward(obj.h, K[P], K[Q], K[R], dY.data_ptr(), d, d,
                                        nat.ptr(ref), EPI[epi], float(slope), dX.data_ptr(), d,
                                        comm, ws.data_ptr(), ws.numel(), _st(dev)),
              "hgd_conv2hop_backward")
    return dX


def test_object_structure_matches_python_incidence(dev):
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    rng = np.random.default_rng(3)
    Nv, Ne = 700, 300
    r, c = random_coo(rng, Nv, Ne, 9000)
    vals = rng.random(len(r)).astype(np.float32) + 0.1
    rowptr, col, rs, cs = _csr_of(r, c, Nv, dev)
    val = torch.from_numpy(vals).to(dev)  # random_coo is row-major sorted: same order
    obj = _create(rowptr, col, val, Nv, Ne, dev)
    inc = Incidence.from_coo(torch.from_numpy(np.stack([r, c])), torch.from_numpy(vals), (Nv, Ne),
                             device=dev)
    v = obj.view()
    assert (v.n_rows, v.n_cols, v.nnz) == (Nv, Ne, len(r))
    nnz = len(r)
    assert torch.equal(_dev_array(v.colptr, Ne + 1, torch.int64, dev), inc.csc.rowptr)
    assert torch.equal(_dev_array(v.row_t, nnz, torch.int32, dev), inc.csc.col)
    assert torch.equal(_dev_array(v.perm_t, nnz, torch.int32, dev), inc.perm_t)
    assert torch.equal(_dev_array(v.val_t, nnz, torch.float32, dev), inc.val_t)
    for side, name in ((0, "row"), (1, "col")):
        for kind in ("mean", "sym", "wmean", "wsym"):
            got = _dev_array(obj.scale(side, kind), Nv if side == 0 else Ne, torch.float32, dev)
            assert torch.equal(got, inc.scale(name, kind)), (name, kind)
    assert obj.scale(0, None) is None


CASES = [
    ("hgconv2", False, "sym", "mean", "sym", None, 0.0),
    ("mean2hop", False, "mean", "mean", None, None, 0.0),
    ("hgcnconv_act", True, None, None, None, "leaky_relu", 0.5),
    ("weighted_sym", True, "wsym", "wmean", "wsym", "relu", 0.0),
    ("neg_slope", True, None, None, None, "leaky_relu", -0.3),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("heavy", [False, True])
def test_conv2hop_matches_two_hop_and_oracle(dev, case, heavy):
    from hypergraph_diffusion_for_recommendation_amd import Incidence, two_hop
    name, weighted, P, Q, R, epi, slope = case
    rng = np.random.default_rng(zlib.crc32(name.encode()) % 997 + heavy)
    Nv, Ne, d = 900, 40, 64
    r, c = random_coo(rng, Nv, Ne, 12000)
    if heavy:  # rows / columns long enough for split plans (auto_split: small row counts)
        extra_r = np.repeat(np.arange(3), Ne)
        extra_c = np.tile(np.arange(Ne), 3)
        key = np.unique(np.concatenate([r * Ne + c, extra_r * Ne + extra_c]))
        r, c = key // Ne, key % Ne
    vals = (rng.random(len(r)).astype(np.float32) + 0.1) if weighted else None
    rowptr, col, _, _ = _csr_of(r, c, Nv, dev)
    obj = _create(rowptr, col, None if vals is None else torch.from_numpy(vals).to(dev), Nv, Ne,
                  dev)
    inc = Incidence.from_coo(torch.from_numpy(np.stack([r, c])),
                             None if vals is None else torch.from_numpy(vals), (Nv, Ne),
                             device=dev)
    X = rng.standard_normal((Nv, d)).astype(np.float32)
    dY = rng.standard_normal((Nv, d)).astype(np.float32)
    Xt = torch.from_numpy(X).to(dev)
    dYt = torch.from_numpy(dY).to(dev)
    Y, M, pre, ws = _conv(obj, P, Q, R, Xt, epi, slope, dev)
    ref_act = (pre if pre is not None else Y) if epi else None
    dX = _conv_bwd(obj, P, Q, R, dYt, ref_act, epi, slope, dev, ws)
    # bitwise the Python autograd op (same kernels, same plans)
    Xg = Xt.clone().requires_grad_(True)
    Yp = two_hop(inc, Xg, P=P, Q=Q, R=R, epilogue=epi, slope=slope)
    (dXp,) = torch.autograd.grad(Yp, Xg, dYt)
    assert torch.equal(Y, Yp.detach()), name
    assert torch.equal(dX, dXp), name
    # and the float64 oracle
    ref = O.two_hop(r, c, vals, (Nv, Ne), X, P, Q, R, epi, slope)
    w = None if vals is None else np.abs(vals)
    mag = O.two_hop(r, c, w, (Nv, Ne), np.abs(X), P=P, Q=Q, R=R)
    assert_close(Y.cpu().numpy(), ref, mag, what=f"{name} fwd")
    Z = O.two_hop(r, c, vals, (Nv, Ne), X, P, Q, R)
    dref = O.two_hop_backward(r, c, vals, (Nv, Ne), Z, dY, P, Q, R, epi, slope)
    dmag = O.two_hop_backward(r, c, w, (Nv, Ne), np.ones_like(ref), np.abs(dY), P, Q, R, None)
    if epi == "leaky_relu":
        dmag = dmag * max(1.0, abs(slope))
    assert_close(dX.cpu().numpy(), dref, dmag, what=f"{name} bwd")
    if heavy:
        from hypergraph_diffusion_for_recommendation_amd import _native
        assert inc.csc.n_heavy > 0  # the plan path was exercised


def test_incidence_spmm_both_orientations(dev):
    nat, lib = _lib()
    rng = np.random.default_rng(11)
    Nv, Ne, d = 500, 200, 32
    r, c = random_coo(rng, Nv, Ne, 5000)
    vals = rng.random(len(r)).astype(np.float32)
    rowptr, col, _, _ = _csr_of(r, c, Nv, dev, shuffle_within_rows=True, rng=rng)
    # shuffled columns inside rows: permute the values the same way
    # (rebuild vals in the shuffled order from a dense lookup)
    dense = np.zeros((Nv, Ne), np.float32)
    dense[r, c] = vals
    rs = np.repeat(np.arange(Nv), np.diff(rowptr.cpu().numpy()))
    cs = col.cpu().numpy()
    val = torch.from_numpy(dense[rs, cs]).to(dev)
    obj = _create(rowptr, col, val, Nv, Ne, dev)
    X = torch.randn(Ne, d, device=dev)
    XT = torch.randn(Nv, d, device=dev)
    ws = torch.empty(max(1, lib.hgd_incidence_workspace_size(obj.h, d)), dtype=torch.uint8,
                     device=dev)
    Y = torch.empty(Nv, d, device=dev)
    YT = torch.empty(Ne, d, device=dev)
    nat.check(lib.hgd_incidence_spmm(obj.h, 0, X.data_ptr(), d, Y.data_ptr(), d, d, None, 0, 0.0,
                                     ws.data_ptr(), ws.numel(), _st(dev)), "spmm")
    nat.check(lib.hgd_incidence_spmm(obj.h, 1, XT.data_ptr(), d, YT.data_ptr(), d, d,
                                     obj.scale(1, "mean"), 0, 0.0, ws.data_ptr(), ws.numel(),
                                     _st(dev)), "spmm^T")
    A = dense.astype(np.float64)
    assert_close(Y.cpu().numpy(), A @ X.cpu().numpy().astype(np.float64),
                 np.abs(A) @ np.abs(X.cpu().numpy().astype(np.float64)), what="A·X")
    deg = (dense != 0).sum(0)
    s = np.where(deg > 0, 1.0 / np.maximum(deg, 1), 0.0)
    refT = s[:, None] * (A.T @ XT.cpu().numpy().astype(np.float64))
    magT = s[:, None] * (np.abs(A.T) @ np.abs(XT.cpu().numpy().astype(np.float64)))
    assert_close(YT.cpu().numpy(), refT, magT, what="mean·Aᵀ·X")


@pytest.mark.parametrize("weighted", [True, False])
def test_dropedge_child(dev, weighted):
    nat, lib = _lib()
    rng = np.random.default_rng(5 + weighted)
    Nv, Ne, d, keep = 600, 250, 64, 0.7
    r, c = random_coo(rng, Nv, Ne, 8000)
    vals = (rng.random(len(r)).astype(np.float32) + 0.1) if weighted else None
    rowptr, col, _, _ = _csr_of(r, c, Nv, dev)
    obj = _create(rowptr, col, None if vals is None else torch.from_numpy(vals).to(dev), Nv, Ne,
                  dev)
    mask = (rng.random(len(r)) < keep).astype(np.uint8)
    m = torch.from_numpy(mask).to(dev)
    h = ctypes.c_void_p()
    nat.check(lib.hgd_incidence_dropedge(obj.h, m.data_ptr(), keep, ctypes.byref(h), _st(dev)),
              "dropedge")
    child = Obj(h.value)
    v = child.view()
    kept = int(mask.sum())
    assert v.nnz == kept and v.perm_t is None
    base = vals if weighted else np.ones(len(r), np.float32)
    idx, nv = O.dropedge(np.stack([r, c]), base, mask.astype(bool), keep)
    got_rp = _dev_array(v.rowptr, Nv + 1, torch.int64, dev).cpu().numpy()
    got_c = _dev_array(v.col, kept, torch.int32, dev).cpu().numpy()
    got_v = _dev_array(v.val, kept, torch.float32, dev).cpu().numpy()
    assert np.array_equal(np.repeat(np.arange(Nv), np.diff(got_rp)), idx[0])
    assert np.array_equal(got_c, idx[1])
    assert np.array_equal(got_v, nv.astype(np.float32))
    # a child conv equals the oracle on the dropped COO; a child cannot be dropped again
    X = rng.standard_normal((Nv, d)).astype(np.float32)
    Y, _, _, _ = _conv(child, None, None, None, torch.from_numpy(X).to(dev), None, 0.0, dev)
    ref = O.two_hop(idx[0], idx[1], nv, (Nv, Ne), X)
    mag = O.two_hop(idx[0], idx[1], np.abs(nv), (Nv, Ne), np.abs(X))
    assert_close(Y.cpu().numpy(), ref, mag, what="child conv")
    h2 = ctypes.c_void_p()
    assert lib.hgd_incidence_dropedge(child.h, m.data_ptr(), keep, ctypes.byref(h2),
                                      _st(dev)) == 3  # HGD_ERR_UNSUPPORTED


def test_from_dense_matches_nonzero(dev):
    nat, lib = _lib()
    g = torch.Generator().manual_seed(2)
    H = torch.randn(300, 48, generator=g)
    H[H.abs() < 0.8] = 0
    Hd = H.to(dev)
    for keep_values in (0, 1):
        h = ctypes.c_void_p()
        nat.check(lib.hgd_incidence_from_dense(Hd.data_ptr(), 300, 48, 48, 0.0, 1, keep_values,
                                               ctypes.byref(h), _st(dev)), "from_dense")
        obj = Obj(h.value)
        v = obj.view()
        nz = torch.nonzero(H)
        assert v.nnz == nz.shape[0]
        rp = _dev_array(v.rowptr, 301, torch.int64, dev).cpu()
        assert torch.equal(torch.repeat_interleave(torch.arange(300), rp[1:] - rp[:-1]), nz[:, 0])
        assert torch.equal(_dev_array(v.col, v.nnz, torch.int32, dev).cpu().long(), nz[:, 1])
        if keep_values:
            assert torch.equal(_dev_array(v.val, v.nnz, torch.float32, dev).cpu(), H[H != 0])
        else:
            assert v.val is None


def test_create_rejects_malformed(dev):
    nat, lib = _lib()
    h = ctypes.c_void_p()
    rowptr = torch.tensor([0, 2, 1, 3], dtype=torch.int64, device=dev)  # decreasing
    col = torch.tensor([0, 1, 2], dtype=torch.int32, device=dev)
    assert lib.hgd_incidence_create(rowptr.data_ptr(), col.data_ptr(), None, 3, 4, 3,
                                    ctypes.byref(h), _st(dev)) == 1
    assert b"malformed" in lib.hgd_get_last_error_string()
    rowptr = torch.tensor([0, 1, 2, 3], dtype=torch.int64, device=dev)
    col = torch.tensor([0, 9, 2], dtype=torch.int32, device=dev)  # column out of range
    assert lib.hgd_incidence_create(rowptr.data_ptr(), col.data_ptr(), None, 3, 4, 3,
                                    ctypes.byref(h), _st(dev)) == 1
    empty = _create(torch.zeros(5, dtype=torch.int64, device=dev),
                    torch.zeros(0, dtype=torch.int32, device=dev), None, 4, 7, dev)
    Y, M, _, _ = _conv(empty, "sym", "mean", "sym", torch.randn(4, 16, device=dev), None, 0.0,
                       dev)
    assert (Y == 0).all() and (M == 0).all()


@pytest.mark.parametrize("blocks", ["0", "3"])
def test_one_rank_comm_matches_local(dev, monkeypatch, blocks):
    """hgd_comm over one rank: globalize leaves the item scales as they were (to rounding of
    the float64 pow), chunked + all-reduced hop 1 equals the local conv — also with the
    source-blocked hop forced (HGD_SPMM_BLOCKS=3: every chunk's rows blocked as the local
    hop's, so still bitwise)."""
    nat, lib = _lib()
    monkeypatch.setenv("HGD_SPMM_BLOCKS", blocks)
    rng = np.random.default_rng(9)
    Nv, Ne, d = 3000, 800, 64
    r, c = random_coo(rng, Nv, Ne, 20000)
    # no CSC row above the auto split threshold (2·32 at this size): the blocked hop applies
    assert np.bincount(c, minlength=Ne).max() <= 64
    rowptr, col, _, _ = _csr_of(r, c, Nv, dev)
    obj = _create(rowptr, col, None, Nv, Ne, dev)
    X = torch.randn(Nv, d, device=dev)
    dY = torch.randn(Nv, d, device=dev)
    Y0, M0, _, ws = _conv(obj, "sym", "mean", "sym", X, None, 0.0, dev)
    dX0 = _conv_bwd(obj, "sym", "mean", "sym", dY, None, None, 0.0, dev, ws)
    q0 = _dev_array(obj.scale(1, "mean"), Ne, torch.float32, dev)
    if blocks != "0":  # the blocked hop was taken: its M differs from the plain hop's in bits
        monkeypatch.setenv("HGD_SPMM_BLOCKS", "0")
        _, Mp, _, _ = _conv(obj, "sym", "mean", "sym", X, None, 0.0, dev)
        assert not torch.equal(Mp, M0)
        monkeypatch.setenv("HGD_SPMM_BLOCKS", blocks)
    uid = ctypes.create_string_buffer(nat.COMM_ID_BYTES)
    nat.check(lib.hgd_comm_get_unique_id(uid), "unique id")
    comm = ctypes.c_void_p()
    nat.check(lib.hgd_comm_create(uid, 1, 0, ctypes.byref(comm)), "comm_create")
    try:
        # a sharded conv needs global item scales first
        assert lib.hgd_conv2hop_forward(obj.h, 2, 1, 2, X.data_ptr(), d, d, Y0.data_ptr(), d, 0,
                                        0.0, None, None, comm, ws.data_ptr(), ws.numel(),
                                        _st(dev)) == 1
        nat.check(lib.hgd_incidence_globalize_columns(obj.h, comm, _st(dev)), "globalize")
        q1 = _dev_array(obj.scale(1, "mean"), Ne, torch.float32, dev)
        assert torch.equal(q0, q1)
        nat.check(lib.hgd_comm_set_chunks(comm, 3), "chunks")
        Y1, M1, _, ws1 = _conv(obj, "sym", "mean", "sym", X, None, 0.0, dev, comm=comm)
        dX1 = _conv_bwd(obj, "sym", "mean", "sym", dY, None, None, 0.0, dev, ws1, comm=comm)
        torch.cuda.synchronize(dev)
        assert torch.equal(M0, M1) and torch.equal(Y0, Y1) and torch.equal(dX0, dX1)
        buf = torch.randn(1000, device=dev)
        ref = buf.clone()
        nat.check(lib.hgd_exchange_allreduce(comm, buf.data_ptr(), buf.numel(), _st(dev)),
                  "allreduce")
        torch.cuda.synchronize(dev)
        assert torch.equal(buf, ref)
    finally:
        lib.hgd_comm_destroy(comm)


@pytest.mark.parametrize("case", [CASES[0], CASES[3]], ids=[CASES[0][0], CASES[3][0]])
def test_conv2hop_source_blocked_matches_python(dev, monkeypatch, case):
    """With HGD_SPMM_BLOCKS forcing the source-blocked hop (hgd_spmm_blocked; the size rule
    picks it only for ≥ 1 GiB tables), the object path blocks its CSC hops exactly as the Python
    Incidence does: conv2hop fwd/bwd and hgd_incidence_spmm(transpose) bitwise equal to
    functional.two_hop / spmm_csr, and the forward within the oracle bound."""
    from hypergraph_diffusion_for_recommendation_amd import Incidence, spmm_csr, two_hop
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_blocks
    nat, lib = _lib()
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "3")
    name, weighted, P, Q, R, epi, slope = case
    rng = np.random.default_rng(71)
    Nv, Ne, d = 3000, 800, 64
    r, c = random_coo(rng, Nv, Ne, 20000)
    vals = (rng.random(len(r)).astype(np.float32) + 0.1) if weighted else None
    rowptr, col, _, _ = _csr_of(r, c, Nv, dev)
    obj = _create(rowptr, col, None if vals is None else torch.from_numpy(vals).to(dev), Nv, Ne,
                  dev)
    inc = Incidence.from_coo(torch.from_numpy(np.stack([r, c])),
                             None if vals is None else torch.from_numpy(vals), (Nv, Ne),
                             device=dev)
    assert inc.csc.n_heavy == 0 and spmm_blocks(inc.csc, d) == 3
    X = rng.standard_normal((Nv, d)).astype(np.float32)
    Xt = torch.from_numpy(X).to(dev)
    dYt = torch.from_numpy(rng.standard_normal((Nv, d)).astype(np.float32)).to(dev)
    Y, M, pre, ws = _conv(obj, P, Q, R, Xt, epi, slope, dev)
    dX = _conv_bwd(obj, P, Q, R, dYt, (pre if pre is not None else Y) if epi else None, epi,
                   slope, dev, ws)
    Xg = Xt.clone().requires_grad_(True)
    Yp = two_hop(inc, Xg, P=P, Q=Q, R=R, epilogue=epi, slope=slope)
    (dXp,) = torch.autograd.grad(Yp, Xg, dYt)
    assert torch.equal(Y, Yp.detach()) and torch.equal(dX, dXp), name
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "0")  # the blocked sums are not the plain ones bitwise
    Y0, _, _, _ = _conv(obj, P, Q, R, Xt, epi, slope, dev)
    assert not torch.equal(Y, Y0)
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "3")
    ref = O.two_hop(r, c, vals, (Nv, Ne), X, P, Q, R, epi, slope)
    w = None if vals is None else np.abs(vals)
    mag = O.two_hop(r, c, w, (Nv, Ne), np.abs(X), P=P, Q=Q, R=R)
    assert_close(Y.cpu().numpy(), ref, mag, what=f"{name} blocked fwd")
    # the transposed plain hop of hgd_incidence_spmm
    Yt = torch.empty(Ne, d, device=dev)
    wsb = lib.hgd_incidence_workspace_size(obj.h, d)
    ws2 = torch.empty(max(1, wsb), dtype=torch.uint8, device=dev)
    nat.check(lib.hgd_incidence_spmm(obj.h, 1, Xt.data_ptr(), d, Yt.data_ptr(), d, d, None, 0,
                                     0.0, ws2.data_ptr(), wsb, _st(dev)), "hgd_incidence_spmm")
    assert torch.equal(Yt, spmm_csr(inc.csc, Xt, val=inc.val_t))
