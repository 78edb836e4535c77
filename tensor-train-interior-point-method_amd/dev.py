"""Device op layer: fp64 tensors on the MI355X, every arithmetic op through libttk (HIP).

PyTorch is used only as the allocator / container (torch.empty, views, H2D of host-generated
random numbers); all arithmetic goes through the C ABI in `include/ttk.h`.

* `einsum(eq, *ops)`: greedy pairwise plan (the reference plans with opt_einsum greedy and
  caches the expression per (equation, shapes), `src/tt_ops.py:22-28`); each pairwise step is
  ONE launch of the offset-table MFMA GEMM (`ttk_gemm_offs`), operands addressed through their
  strides, so transposed/permuted views cost nothing.  Plans (offset tables in HBM, intermediate
  buffers) are cached per (equation, shapes, strides).
* small dense factorisations (`svd`, `qr`, `rq`, `cholesky_`, `lu_`, `syev`), reductions and
  strided element-wise kernels.
"""
import ctypes
import os
import threading
from functools import lru_cache

import numpy as np
import torch

from ._lib import LinAlgError, LinAlgWarning, c_dp, c_i64p, check, lib, lib_release

DEV = torch.device(os.environ.get("TTIPM_DEVICE", "cuda"))
F64 = torch.float64
_vp = ctypes.c_void_p


class _PerThread(threading.local):
    """Per-host-thread state of the path: several solves may run at once in one process, one per
    thread, each with its own HIP stream and libttk context (bench.py's solves in flight)."""

    def __init__(self):
        self.stream = []  # the launch stream (the thread's current torch stream when first used)
        self.ctx = []     # the ttk_ctx bound to this thread (created with the stream)
        self.batch = [0]  # open einsum batches (dev.einsum_batch)
        # operands of recorded (not yet launched) einsum steps: held until the flush so that the
        # caching allocator cannot hand their memory to an allocation whose kernels run before them
        self.keep = []
        self.fast = None  # _ttkbind bound to this thread's stream
        self.ones = {}    # small constant device tensors made on this thread's stream
        self.anti = {}
        self.consts = {}  # tt_ops._const's constant cores


_TL = _PerThread()


def ctx():
    """This thread's ttk_ctx handle (None before the first launch)."""
    c = _TL.ctx
    return c[0] if c else None


def _stream():
    """The launch stream (the thread's current stream when first used; the path never switches
    streams, and torch.cuda.current_stream() costs ~10 us per call)."""
    tl = _TL
    if not tl.stream:
        tl.stream.append(torch.cuda.current_stream().cuda_stream if DEV.type == "cuda" else None)
        if DEV.type == "cuda":  # this thread's libttk context: the launch stream + all scratch state
            h = ctypes.c_void_p(0)
            check(lib.ttk_ctx_create(tl.stream[0], ctypes.byref(h)), "ctx_create")
            tl.ctx.append(h)
            check(lib.ttk_ctx_bind(h), "ctx_bind")
    if tl.batch[0]:  # any launch other than an einsum first flushes the recorded steps (stream order)
        check(lib.ttk_einsum_batch_flush(tl.stream[0]), "einsum_batch_flush")
        tl.keep.clear()
    return tl.stream[0]


class einsum_batch:
    """`with dev.einsum_batch(): ...` -- the einsum calls inside are recorded and launched at the end
    as grouped launches, one per dependency level (ttk_einsum_batch_*, bit-identical results).
    Other device operations inside the block stay correct (they flush the pending steps first) but
    split the batch, so keep batch bodies to einsums and fresh allocations."""

    def __enter__(self):
        if DEV.type == "cuda":
            _stream()
            tl = _TL
            check(lib.ttk_einsum_batch_begin(tl.stream[0]), "einsum_batch_begin")
            tl.batch[0] += 1
        return self

    def __exit__(self, *exc):
        if DEV.type == "cuda":
            tl = _TL
            tl.batch[0] -= 1
            check(lib.ttk_einsum_batch_end(tl.stream[0]), "einsum_batch_end")
            if not tl.batch[0]:
                tl.keep.clear()
        return False


def _p(t):
    return t.data_ptr()


def _load_bind():
    """`_ttkbind` (csrc/ttk_host_bind.cpp): packs tensor pointers/shapes/strides natively for the
    hot einsum / copy / mul entry points (same libttk calls; ~8 us of Python packing saved per call)."""
    import glob
    import importlib.util
    if os.environ.get("TTIPM_NO_BIND") == "1":
        return None
    paths = glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ttkbind*.so"))
    if not paths:
        return None
    try:
        spec = importlib.util.spec_from_file_location("_ttkbind", paths[0])
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    except Exception as e:  # same libttk calls through ctypes packing (slower host side)
        import sys
        print(f"ttipm_amd: _ttkbind not loadable ({e}); packing einsum/copy arguments in Python", file=sys.stderr)
        return None
    return mod


_BIND = _load_bind()
if _BIND is not None and os.environ.get("TTK_HOLD_GIL", "1") == "1" and hasattr(_BIND, "set_release_gil"):
    _BIND.set_release_gil(False)  # as the launch-only libttk entry points (_lib.py)


def _fast():
    """_ttkbind bound to this thread's stream (the binder keeps one stream per host thread)."""
    tl = _TL
    if tl.fast is None and _BIND is not None:
        def addr(f):
            return ctypes.cast(f, ctypes.c_void_p).value
        _BIND.bind(addr(lib.ttk_einsum), addr(lib.ttk_copy_nd), addr(lib.ttk_mul_nd), _stream() or 0)
        if _FAST2:
            _BIND.bind2(addr(lib.ttk_axpby_nd), addr(lib.ttk_normalize), addr(lib.ttk_scale_axis_ss),
                        addr(lib.ttk_dot_nd_dev), addr(lib.ttk_fill))
        tl.fast = _BIND
    return tl.fast


_LIKE = []
_BIND_EMPTY = getattr(_BIND, "empty", None)
_FAST2 = hasattr(_BIND, "bind2")  # native packers of axpby / normalized / scale_axis_ss / dot_into / zeros
_COLS = hasattr(_BIND, "einsum_cols")


def _like():
    """a float64 tensor on DEV whose options `_ttkbind.empty` copies"""
    if not _LIKE:
        _LIKE.append(torch.empty(1, dtype=F64, device=DEV))
    return _LIKE[0]


def empty(*shape):
    """a new float64 device tensor (the caching allocator, the thread's current stream).  Through
    _ttkbind when built: at::empty with the GIL held, ~1 us instead of torch.empty's ~3 us, and no
    GIL hand-over to a second solve thread on every allocation (tools/gil_bench.py)."""
    if _BIND_EMPTY is not None and DEV.type == "cuda":
        return _BIND_EMPTY(_like(), shape)
    return torch.empty(shape, dtype=F64, device=DEV)


def zeros(*shape):
    """a zero-filled device tensor: libttk's fill kernel on the launch stream (torch.zeros would
    dispatch its own fill kernel through the torch runtime, ~3x the host cost)"""
    if _FAST2 and DEV.type == "cuda":
        return (_TL.fast or _fast()).zeros(_like(), shape)
    out = empty(*shape)
    if DEV.type == "cuda" and out.numel():
        check(lib.ttk_fill(_stream(), out.data_ptr(), out.numel(), 0.0), "fill")
    elif DEV.type != "cuda":
        out.zero_()
    return out


def from_numpy(a):
    """Host array -> new device tensor, copied asynchronously on the launch stream through libttk's
    pinned upload ring (a pageable torch copy would drain the stream; torch's pin_memory path
    measured ~120 us per call)."""
    h = np.array(a, dtype=np.float64, order="C", copy=True)
    if DEV.type != "cuda":
        return torch.from_numpy(h).to(DEV)
    out = empty(*h.shape)
    if h.size:
        check(lib.ttk_upload(_stream(), h.ctypes.data, out.data_ptr(), h.size), "upload")
    return out


def contig(t):
    """t if contiguous, else a contiguous copy made by the HIP copy kernel (never torch)."""
    return t if t.is_contiguous() else clone(t)


def to_numpy(t):
    return t.detach().to("cpu").numpy()


# optional op statistics (TTIPM_OPSTATS=1): name -> {shape: [count, seconds]} (synchronised timing)
OPSTATS = {} if os.environ.get("TTIPM_OPSTATS") else None


def _stat(name, shape, t0, site_min=None):
    import time as _t
    torch.cuda.synchronize()
    d = OPSTATS.setdefault(name, {})
    e = d.setdefault(shape, [0, 0.0])
    e[0] += 1
    dt = _t.perf_counter() - t0
    e[1] += dt
    if site_min is not None and site_min:  # record the Python call chain of large calls
        import traceback
        chain = " < ".join(f"{f.name}:{f.lineno}" for f in traceback.extract_stack()[-8:-2][::-1])
        s = OPSTATS.setdefault(name + "@sites", {}).setdefault(chain, [0, 0.0])
        s[0] += 1
        s[1] += dt


def _tic():
    import time as _t
    if OPSTATS is not None:
        torch.cuda.synchronize()
    return _t.perf_counter()


def _arr(vals):
    a = (ctypes.c_int64 * len(vals))(*vals)
    return a


# ------------------------------------------------------------------------ element-wise
def copy_(dst, src, alpha=1.0, beta=0.0):
    """dst = alpha * src + beta * dst (shapes must match; any strides)."""
    f = _TL.fast or _fast()
    if f is not None:
        return f.copy_(dst, src, float(alpha), float(beta))
    assert tuple(dst.shape) == tuple(src.shape), (dst.shape, src.shape)
    nd = dst.dim()
    if nd == 0:
        dst = dst.reshape(1)
        src = src.reshape(1)
        nd = 1
    shp = _arr(dst.shape)
    check(lib.ttk_copy_nd(_stream(), _p(src), _p(dst), nd, shp, _arr(src.stride()), _arr(dst.stride()),
                          float(alpha), float(beta)), "copy_nd")
    return dst


def scaled(src, alpha):
    out = empty(*src.shape)
    return copy_(out, src, alpha, 0.0)


def clone(src):
    out = empty(*src.shape)
    return copy_(out, src)


def clone_many(srcs):
    """[clone(t) for t in srcs] as ONE allocation and ONE launch (ttk_copy_many) when every source
    is contiguous (exact copies; the clones are views of one buffer)."""
    n = len(srcs)
    if n < 2 or DEV.type != "cuda" or not all(t.is_contiguous() for t in srcs):
        return [clone(t) for t in srcs]
    counts = [t.numel() for t in srcs]
    buf = empty(sum(counts))
    outs, o = [], 0
    for t, c in zip(srcs, counts):
        outs.append(buf[o:o + c].view(t.shape))
        o += c
    check(lib.ttk_copy_many(_stream(), n, (ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs]),
                            (ctypes.c_void_p * n)(*[t.data_ptr() for t in outs]), (ctypes.c_int64 * n)(*counts)),
          "copy_many")
    return outs


def mul_(dst, a, b, alpha=1.0, beta=0.0):
    """dst = alpha * a * b + beta * dst (element-wise, same shapes, any strides)."""
    f = _TL.fast or _fast()
    if f is not None:
        return f.mul_(dst, a, b, float(alpha), float(beta))
    nd = dst.dim()
    check(lib.ttk_mul_nd(_stream(), _p(a), _p(b), _p(dst), nd, _arr(dst.shape), _arr(a.stride()),
                         _arr(b.stride()), _arr(dst.stride()), float(alpha), float(beta)), "mul_nd")
    return dst


def scale_axis(src, axis, scales, out=None):
    """out = src * scales[i] along `axis` (host scales, <= 16; no H2D copy)."""
    out = empty(*src.shape) if out is None else out
    nd = src.dim()
    sc = (ctypes.c_double * 16)(*[float(v) for v in scales])
    check(lib.ttk_scale_axis(_stream(), _p(src), _p(out), nd, _arr(src.shape), _arr(src.stride()), _arr(out.stride()),
                             int(axis), sc), "scale_axis")
    return out


def axpby(src, src2, alpha, beta, gamma, out=None):
    """out = alpha * src + beta * (gamma * src2) (same shapes, any strides), one launch; rounds like
    scaled(src2, gamma) followed by copy_(out, src, alpha, beta)."""
    if _FAST2 and DEV.type == "cuda":
        return (_TL.fast or _fast()).axpby(src, src2, float(alpha), float(beta), float(gamma), out)
    out = empty(*src.shape) if out is None else out
    nd = src.dim()
    check(lib.ttk_axpby_nd(_stream(), _p(src), _p(src2), _p(out), nd, _arr(src.shape), _arr(src.stride()),
                           _arr(src2.stride()), _arr(out.stride()), float(alpha), float(beta), float(gamma)), "axpby")
    return out


def scale_axis_ss(src, axis, ss, invert, out=None):
    """src * max(sqrt(ss), 1e-10)[i] (or its reciprocal) along `axis`; ss = device sums of squares;
    into `out` (same shape, any strides) when given."""
    if _FAST2 and DEV.type == "cuda":
        return (_TL.fast or _fast()).scale_axis_ss(src, int(axis), ss, bool(invert), out)
    out = empty(*src.shape) if out is None else out
    nd = src.dim()
    check(lib.ttk_scale_axis_ss(_stream(), _p(src), _p(out), nd, _arr(src.shape), _arr(src.stride()),
                                _arr(out.stride()), int(axis), _p(ss), int(bool(invert))), "scale_axis_ss")
    return out


def normalized(src):
    """src / ||src|| as a new contiguous tensor, computed on the device (no host sync)."""
    if _FAST2 and DEV.type == "cuda":
        return (_TL.fast or _fast()).normalized(src)
    out = empty(*src.shape)
    nd = src.dim()
    if nd == 0:
        src, nd = src.reshape(1), 1
    check(lib.ttk_normalize(_stream(), _p(src), _p(out), nd, _arr(src.shape), _arr(src.stride())), "normalize")
    return out


def rayleigh_tail_(v, Mv):
    """ev = <v, Mv>; Mv -= ev v (in place); returns (ev, ||Mv||) with one host read."""
    assert v.is_contiguous() and Mv.is_contiguous() and v.numel() == Mv.numel()
    ev, r2 = ctypes.c_double(0.0), ctypes.c_double(0.0)
    check(lib.ttk_rayleigh_tail_sync(_stream(), _p(v), _p(Mv), v.numel(), ctypes.byref(ev), ctypes.byref(r2)),
          "rayleigh_tail")
    return ev.value, float(np.sqrt(max(r2.value, 0.0)))


def rayleigh_tail_into(v, Mv, out2):
    """ev = <v, Mv>; Mv -= ev v; (ev, ||Mv||^2) -> device out2 (2 doubles), no host wait."""
    assert v.is_contiguous() and Mv.is_contiguous() and v.numel() == Mv.numel() and out2.is_contiguous()
    check(lib.ttk_rayleigh_tail_dev(_stream(), _p(v), _p(Mv), v.numel(), _p(out2)), "rayleigh_tail_dev")


def recip(src):
    src = src.contiguous()
    out = empty(*src.shape)
    check(lib.ttk_recip(_stream(), _p(src), _p(out), src.numel()), "recip")
    return out


def fill_(dst, v):
    assert dst.is_contiguous()
    check(lib.ttk_fill(_stream(), _p(dst), dst.numel(), float(v)), "fill")
    return dst


def add_diag_(A, v):
    check(lib.ttk_add_diag(_stream(), _p(A), A.shape[0], A.stride(0), float(v)), "add_diag")
    return A


def dot(x, y):
    """sum(x*y) over all elements (same shapes), returned to the host."""
    assert tuple(x.shape) == tuple(y.shape)
    nd = x.dim()
    out = ctypes.c_double(0.0)
    if nd == 0:
        x, y, nd = x.reshape(1), y.reshape(1), 1
    check(lib.ttk_dot_nd_sync(_stream(), _p(x), _p(y), nd, _arr(x.shape), _arr(x.stride()), _arr(y.stride()),
                              ctypes.byref(out)), "dot")
    return out.value


def norm(x):
    return float(np.sqrt(max(dot(x, x), 0.0)))


def dot_into(x, y, out):
    """sum(x*y) into the device scalar `out` (a 1-element view), no host synchronisation."""
    if _FAST2 and DEV.type == "cuda":
        return (_TL.fast or _fast()).dot_into(x, y, out)
    assert tuple(x.shape) == tuple(y.shape)
    nd = x.dim()
    if nd == 0:
        x, y, nd = x.reshape(1), y.reshape(1), 1
    check(lib.ttk_dot_nd_dev(_stream(), _p(x), _p(y), nd, _arr(x.shape), _arr(x.stride()), _arr(y.stride()),
                             _p(out)), "dot_into")


def rank_scan(res, negs):
    """res <- res - negs[q] for q in order, <res, res> after each (one launch, one read); the
    per-candidate copy_(res, neg, -1, 1) + dot(res, res) of the rank loop, bit for bit."""
    assert res.is_contiguous() and negs.is_contiguous() and tuple(negs.shape[1:]) == tuple(res.shape)
    nq = negs.shape[0]
    out = np.empty(nq)
    if nq:
        check(lib.ttk_rank_scan_sync(_stream(), _p(res), _p(negs), res.numel(), nq, out.ctypes.data_as(c_dp)),
              "rank_scan")
    return out


def norm_of(d):
    """dev.norm's host formula applied to a read-back <x, x>."""
    return float(np.sqrt(max(float(d), 0.0)))


def read(t):
    """Copy a (small) device tensor to a host numpy array (blocking)."""
    t = t.contiguous()
    out = np.empty(t.shape, dtype=np.float64)
    if t.numel():
        check(lib.ttk_read_sync(_stream(), _p(t), out.ctypes.data_as(c_dp), t.numel()), "read")
    return out


def check_handoffs():
    """Raise if an in-launch hand-off wait of this thread's context gave up since the last check
    (ttk_common.h dep_wait: after DEP_SPIN_MAX polls it counts a timeout and reads on, so the
    one-launch Schur matvec / Arnoldi step / split-K reduce would have used stale words).  One
    stream synchronisation; called once per solve (tt_ipm.tt_ipm) and by the kernel tests."""
    if DEV.type != "cuda" or ctx() is None:
        return
    _stream()
    n = ctypes.c_uint(0)
    check(lib.ttk_dep_timeouts(ctypes.byref(n), 1), "dep_timeouts")
    if n.value:
        raise RuntimeError(f"{n.value} in-launch hand-off wait(s) timed out: results of this solve are invalid")


# ------------------------------------------------------------------------ einsum planner
def _ones_buf():
    t = _TL.ones.get("o")
    if t is None:
        t = torch.ones(1, dtype=F64, device=DEV)
        _TL.ones["o"] = t
    return t


def _parse(eq):
    eq = eq.replace(" ", "")
    lhs, out = eq.split("->")
    return lhs.split(","), out


@lru_cache(maxsize=None)
def _eq_bytes(eq):
    return eq.encode()


@lru_cache(maxsize=65536)
def _out_shape(eq, shapes):
    ins, out = _parse(eq)
    ext = {}
    for idx, shp in zip(ins, shapes):
        for c, e in zip(idx, shp):
            ext[c] = e
    return tuple(ext[c] for c in out)


_CHECK_FUSED = os.environ.get("TTIPM_CHECK_FUSED") == "1"
_FUSED_EQS = ("lsr,smnS,LSR,rnR->lmL", "lsr,smnS,LSR,lmL->rnR")
CHECK_LOG = []


def _einsum_checked(eq, ops, out, alpha, beta):
    """dev diagnostics: run a fused-kernel equation both ways and record the discrepancy"""
    ref_out = None if out is None else clone(out)
    old_host = None if out is None else read(out)
    res = _einsum_native(eq, *ops, out=out, alpha=alpha, beta=beta, fused=True)
    old = lib.ttk_einsum_set_fused(0)
    try:
        plain = _einsum_native(eq, *ops, out=ref_out, alpha=alpha, beta=beta)
    finally:
        lib.ttk_einsum_set_fused(old)
    a, b = read(res), read(plain)
    # error relative to the magnitude of the summed terms (|P| |A| |Q| |x|), not of the result: the
    # local operator cancels to rounding noise on converged directions
    mag = np.einsum(eq, *[np.abs(read(o)) for o in ops], optimize="greedy") * abs(alpha)
    err = float(np.max(np.abs(a - b))) / max(float(np.max(mag)), 1e-300) if b.size else 0.0
    if err > 1e-8 and sum(1 for e in CHECK_LOG if e[-1] > 1e-8) < 4:
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez(f"gpurun_out/fused_bad_{len(CHECK_LOG)}.npz", *[read(o) for o in ops], fused=a, plain=b,
                 old=old_host if old_host is not None else np.zeros(0), eq=np.array(eq), beta=np.array(beta), alpha=np.array(alpha))
    def span(t):
        return t.data_ptr(), t.data_ptr() + 8 * (1 + sum((e - 1) * st for e, st in zip(t.shape, t.stride())))

    overlap = None
    if out is not None:
        o0, o1 = span(out)
        overlap = [k for k, o in enumerate(ops) if span(o)[0] < o1 and o0 < span(o)[1]]
    CHECK_LOG.append((overlap, eq, tuple(tuple(o.shape) for o in ops), tuple(tuple(o.stride()) for o in ops),
                      None if out is None else (tuple(out.shape), tuple(out.stride())), alpha, beta, err))
    return res


_FUSED_ALL = os.environ.get("TTIPM_FUSED_ALL") == "1"  # experiment switch: every local apply fused


# Algorithmic contraction FLOPs: when ALGO is a dict, every einsum call adds the
# FLOP count of the pairwise greedy path for its equation and shapes (opt_einsum's convention, which
# the oracle's counter restates at the reference's call sites), whatever plan (fused launch, pairwise
# MFMA GEMMs) the device executes.  Operator applications made natively (Schur
# handle, LGMRES chunks) are added by their callers with `count_algo`.
ALGO = None
_ALGO_CACHE = {}


def algo_flops(eq, shapes):
    f = _ALGO_CACHE.get((eq, shapes))
    if f is None:
        import re
        # pairwise greedy without NumPy's default intermediate-size cap (opt_einsum's greedy has none;
        # the capped planner collapses 4-operand chains into one naive contraction)
        txt = np.einsum_path(eq, *[np.empty(sh) for sh in shapes], optimize=("greedy", 1 << 62))[1]
        f = float(re.search(r"Optimized FLOP count:\s*([0-9.eE+-]+)", txt).group(1))
        _ALGO_CACHE[(eq, shapes)] = f
    return f


def count_algo(flops, calls=1, what=None):
    if ALGO is not None:
        ALGO["flops"] += flops
        ALGO["calls"] += calls
        if what is not None and "by" in ALGO:
            e = ALGO["by"].setdefault(what, [0, 0.0])
            e[0] += calls
            e[1] += flops


def einsum(eq, *ops, out=None, alpha=1.0, beta=0.0, fused=False, algo=None):
    """`fused=True` lets the local-operator equations run as one fused launch (see ttk_einsum);
    call sites whose results feed noise-level decisions keep the pairwise plan.  `fused="env"`:
    a relabelled environment update (fused under a smaller FLOP limit).  `algo=(eq, shapes)`: the
    reference's own equation and operand shapes for a relabelled call, so the algorithmic count
    follows the reference's contraction order."""
    if ALGO is not None:
        if algo is not None:
            count_algo(algo_flops(*algo), what=algo[0])
        else:
            count_algo(algo_flops(eq, tuple(tuple(o.shape) for o in ops)), what=eq)
    fused = fused or _FUSED_ALL
    tl = _TL
    if tl.batch[0]:
        if out is None:
            out = _new_out(eq, ops)
            beta = 0.0
        tl.keep.append((ops, out))
    if _CHECK_FUSED and fused and eq in _FUSED_EQS:
        return _einsum_checked(eq, ops, out, alpha, beta)
    return _einsum_native(eq, *ops, out=out, alpha=alpha, beta=beta, fused=fused)


def einsum_cols(eqs, items, x, out, alpha=1.0, beta=1.0):
    """A run of einsums over block columns: item = (equation index into `eqs`, operands, x column or
    -1, out column) computes out[:, ocol] = alpha * einsum(eq, *operands, x[:, xcol]) + beta *
    out[:, ocol], in item order.  One native call (`_ttkbind.einsum_cols`: the same libttk einsum
    calls, in the same order, as one `einsum` per item) instead of a Python slice and wrapper per
    block; the per-item path when FLOPs are being counted or the native packer is absent."""
    f = _TL.fast or _fast()
    if f is None or not _COLS or ALGO is not None or OPSTATS is not None or _CHECK_FUSED:
        for ei, ops, xc, oc in items:
            einsum(eqs[ei], *ops, *((x[:, xc],) if xc >= 0 else ()), out=out[:, oc], alpha=alpha, beta=beta)
        return out
    tl = _TL
    if tl.batch[0]:
        tl.keep.append((items, x, out))
    f.einsum_cols(eqs, items, x, out, float(alpha), float(beta), 256 if _FUSED_ALL else 0)
    return out


def _new_out(eq, ops):
    return empty(*_out_shape(eq, tuple(tuple(o.shape) for o in ops)))


def _einsum_native(eq, *ops, out=None, alpha=1.0, beta=0.0, fused=False):
    """out = alpha * einsum(eq, *ops) + beta * out, on the device.  Planning (greedy pairwise
    order, offset tables) and execution (one fp64 MFMA GEMM launch per pairwise step) happen in
    the native engine `ttk_einsum` (csrc/ttk_einsum.hip); this wrapper only packs pointers,
    shapes and strides."""
    if OPSTATS is not None:
        e = OPSTATS.setdefault("einsum_eq", {}).setdefault(eq, [0, 0.0])
        e[0] += 1
    f = _TL.fast or _fast()
    if f is not None:
        return f.einsum(eq, ops, out, float(alpha), float(beta), (256 | 512) if fused == "env" else (256 if fused else 0))
    desc = [len(ops) | ((256 | 512) if fused == "env" else (256 if fused else 0))]
    for o in ops:
        desc.append(o.data_ptr())
        desc.append(o.dim())
        desc.extend(o.shape)
        desc.extend(o.stride())
    if out is None:
        out = empty(*_out_shape(eq, tuple(tuple(o.shape) for o in ops)))
        beta = 0.0
        desc.append(0)
    else:
        desc.append(1)
        desc.append(out.dim())
        desc.extend(out.stride())
    st = _TL.stream[0] if _TL.stream else _stream()  # no batch flush: einsums are recorded
    check(lib.ttk_einsum(st, _eq_bytes(eq), (ctypes.c_int64 * len(desc))(*desc), out.data_ptr(),
                         float(alpha), float(beta)), "einsum")
    return out


def apply_desc(P, A, Q, xshape):
    """ttk_einsum descriptor of the local apply 'lsr,smnS,LSR,rnR->lmL' with operands P, A, Q and a
    placeholder x of shape `xshape` (pointer patched per call by ttk_schur_apply); 36 words."""
    d = [4 | 256]
    for o in (P, A, Q):
        d.append(o.data_ptr())
        d.append(o.dim())
        d.extend(o.shape)
        d.extend(o.stride())
    r, n, R = xshape
    d.extend([0, 3, r, n, R, n * R, R, 1, 0])
    return d


def tensordot(a, b, axes):
    """numpy-style tensordot via the einsum executor."""
    ax_a, ax_b = axes
    letters = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
    ia = list(letters[:a.dim()])
    ib = list(letters[a.dim():a.dim() + b.dim()])
    for x, y in zip(ax_a, ax_b):
        ib[y] = ia[x]
    outi = [c for i, c in enumerate(ia) if i not in ax_a] + [c for i, c in enumerate(ib) if i not in ax_b]
    return einsum("".join(ia) + "," + "".join(ib) + "->" + "".join(outi), a, b)


def matmul(a, b, out=None, alpha=1.0, beta=0.0):
    return einsum("ik,kj->ij", a, b, out=out, alpha=alpha, beta=beta)


# ------------------------------------------------------------------------ factorisations
_DUMP = {"min": int(os.environ.get("TTIPM_DUMP_SVD", "0")), "max": int(os.environ.get("TTIPM_DUMP_SVD_MAX", "1000000")),
         "qmin": int(os.environ.get("TTIPM_DUMP_SVD_QMIN", "0")), "n": 0}


_SVD_READ = hasattr(lib, "ttk_svd_tol_read")  # False only for an older library under TTK_LIB_PATH


def svd(A, defl=0.0, host=True, S_out=None):
    """Thin SVD of a 2-D device matrix.  Returns (U, S, Vt, s_host).  `defl` > 0 lets the large-
    matrix path deflate directions whose total Frobenius norm is <= defl (S = 0 there).
    host=False: no host copy of S (s_host None), so the call does not synchronise.  `S_out`: a
    contiguous device slice of length min(m, n) that receives S (to be read together with other
    device scalars in one host wait)."""
    t0 = _tic() if OPSTATS is not None else 0
    A = A.contiguous()
    m, n = A.shape
    if _DUMP["min"] and _DUMP["min"] <= min(m, n) <= _DUMP["max"] and max(m, n) >= _DUMP["qmin"] \
            and _DUMP["n"] < 12:  # dev diagnostics only
        os.makedirs("gpurun_out", exist_ok=True)
        np.save(f"gpurun_out/svd_in_{_DUMP['n']}.npy", read(A))
        _DUMP["n"] += 1
    k = min(m, n)
    U, S, Vt = empty(m, k), (empty(k) if S_out is None else S_out), empty(k, n)
    work = empty(int(lib.ttk_svd_work(m, n)))
    # p > 96 takes the multi-launch path (host loops over Jacobi rounds): release the GIL meanwhile
    L = lib_release if min(m, n) > 96 else lib
    if host and _SVD_READ:  # the SVD and the host read of S in one call (the kernel stores S itself)
        sh = np.empty(k, dtype=np.float64)
        check(lib.ttk_svd_tol_read(_stream(), _p(A), m, n, _p(U), _p(S), _p(Vt), _p(work), float(defl),
                                 sh.ctypes.data_as(c_dp)), "svd")
    else:
        check(L.ttk_svd_tol(_stream(), _p(A), m, n, _p(U), _p(S), _p(Vt), _p(work), float(defl)), "svd")
        sh = read(S) if host else None
    if OPSTATS is not None:
        _stat("svd", (m, n), t0, site_min=min(m, n) >= 64)
    return U, S, Vt, sh


def qr(A):
    """Economic Householder QR: A (m,n) = Q (m,k) R (k,n)."""
    t0 = _tic() if OPSTATS is not None else 0
    A = A.contiguous()
    m, n = A.shape
    k = min(m, n)
    Q, R = empty(m, k), empty(k, n)
    work = empty(int(lib.ttk_qr_work(m, n)))
    L = lib_release if min(m, n) >= 48 else lib  # the blocked path's host loop over panels
    check(L.ttk_qr(_stream(), _p(A), m, n, _p(Q), _p(R), _p(work)), "qr")
    if OPSTATS is not None:
        _stat("qr", (m, n), t0, site_min=min(m, n) >= 64)
    return Q, R


def _anti_identity(n):
    t = _TL.anti.get(n)
    if t is None:
        t = from_numpy(np.eye(n)[::-1])
        _TL.anti[n] = t
    return t


def rq(M):
    """Economic RQ (scipy.linalg.rq mode='economic') via QR of the row-reversed transpose:
    M = R Q with Q orthonormal rows; J = anti-identity, M^T J = Qt Rt  =>  R = J Rt^T J, Q = J Qt^T."""
    p, q = M.shape
    k = min(p, q)
    Jp, Jk = _anti_identity(p), _anti_identity(k)
    Qt, Rt = qr(einsum("ji,jk->ik", M, Jp))
    R = einsum("ij,lj,lk->ik", Jp, Rt, Jk)
    Q = einsum("ij,lj->il", Jk, Qt)
    return R, Q


def cholesky_(A):
    """In-place lower Cholesky; raises LinAlgError if not positive definite."""
    assert A.is_contiguous()
    check(lib.ttk_cholesky_sync(_stream(), _p(A), A.shape[0]), "cholesky")
    return A


def trsm_(L, B, trans=False):
    """B <- op(L)^{-1} B in place (L lower, row-major contiguous); B (n, nrhs) row-major."""
    assert L.is_contiguous() and B.stride(1) == 1
    check(lib.ttk_trsm_lower(_stream(), _p(L), L.shape[0], _p(B), B.shape[1], B.stride(0), int(trans)), "trsm")
    return B


_EPS_E = float(np.finfo(np.float64).eps) / 2  # LAPACK dlamch('E')


def lu_(A, check_rcond=True):
    """In-place getrf; returns pivots.  Raises LinAlgError on an exact zero pivot and, like
    scipy.linalg.solve under warnings-as-errors, LinAlgWarning when rcond < eps."""
    assert A.is_contiguous()
    n = A.shape[0]
    piv = torch.empty(n, dtype=torch.int32, device=DEV)
    work = empty(2 * n + 16)
    rc = ctypes.c_double(0.0)
    check(lib.ttk_lu_sync(_stream(), _p(A), n, _p(piv), _p(work), ctypes.byref(rc)), "lu")
    if check_rcond and rc.value < _EPS_E:
        raise LinAlgWarning(f"Ill-conditioned matrix (rcond={rc.value:.5g}): result may not be accurate.")
    return piv


def lu_solve_(LU, piv, B):
    assert B.stride(-1) == 1
    B2 = B.reshape(B.shape[0], -1)
    check(lib.ttk_lu_solve(_stream(), _p(LU), LU.shape[0], _p(piv), _p(B2), B2.shape[1], B2.stride(0)), "lu_solve")
    return B


def syev(A):
    """Symmetric eigen-decomposition (Jacobi).  Returns (ev device, W device, ev_host)."""
    t0 = _tic() if OPSTATS is not None else 0
    A = clone(A)
    n = A.shape[0]
    ev, W = empty(n), empty(n, n)
    work = empty(int(lib.ttk_syev_work(n)))
    check(lib_release.ttk_syev(_stream(), _p(A), n, _p(ev), _p(W), _p(work)), "syev")
    evh = read(ev)
    if OPSTATS is not None:
        _stat("syev", n, t0)
    return ev, W, evh


def syev_extreme(A, largest=False, lam_out=None):
    """One extreme eigenpair of a symmetric device matrix (Householder tridiagonalisation +
    multisection + inverse iteration, one launch).  Returns (eigenvalue float, unit vector); with
    `lam_out` (a device slice of length 1) the eigenvalue stays there and is not read: (None, vector)."""
    t0 = _tic() if OPSTATS is not None else 0
    A = A.contiguous()
    n = A.shape[0]
    buf = empty(n + 1) if lam_out is None else None
    lam_p, vec = (buf[:1], buf[1:]) if lam_out is None else (lam_out, empty(n))
    work = empty(int(lib.ttk_syev_extreme_work(n)))
    # n > 128: one launch per Householder reflector from the host -- release the GIL meanwhile
    L = lib_release if n > 128 else lib
    check(L.ttk_syev_extreme(_stream(), _p(A), n, 1 if largest else 0, _p(lam_p), _p(vec), _p(work)),
          "syev_extreme")
    if lam_out is not None:
        return None, vec
    lam = float(read(buf[:1])[0])
    if OPSTATS is not None:
        _stat("syev_extreme", n, t0, site_min=n >= 200)
    return lam, buf[1:]


__all__ = ["axpby", "scale_axis_ss", "dot_into", "norm_of", "normalized", "rayleigh_tail_", "scale_axis", "syev_extreme", "einsum", "tensordot", "matmul", "copy_", "scaled", "clone", "mul_", "recip", "fill_", "add_diag_",
           "dot", "norm", "read", "svd", "qr", "rq", "cholesky_", "trsm_", "lu_", "lu_solve_", "syev", "empty",
           "zeros", "from_numpy", "to_numpy", "LinAlgError", "LinAlgWarning"]
