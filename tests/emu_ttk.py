"""NumPy emulation of the libttk C ABI -- TEST INFRASTRUCTURE for CPU-only tests.

Lets the `-m "not gpu"` suite exercise the product's HOST logic (einsum planner, TT algebra,
AMEn / IPM control flow, LGMRES bookkeeping) on CPU tensors, by swapping `ttipm_amd._lib.lib`
for this object before `ttipm_amd.dev` is imported (see `emulated_ttipm()` below).  It is
never used by the product, by `smoke()` or by `bench.py`; the GPU tests run the real HIP
library and fail if it is missing."""
import ctypes
import importlib
import os
import sys

import numpy as np
import scipy.linalg as sla


def _dv(ptr, n):
    if n <= 0:
        return np.zeros(0)
    return np.ctypeslib.as_array((ctypes.c_double * int(n)).from_address(int(ptr)))


def _iv(ptr, n):
    return np.ctypeslib.as_array((ctypes.c_int64 * int(n)).from_address(int(ptr)))


def _i32(ptr, n):
    return np.ctypeslib.as_array((ctypes.c_int32 * int(n)).from_address(int(ptr)))


def _nd_index(ndim, shape, strides):
    shape = [int(shape[i]) for i in range(ndim)]
    idx = np.zeros(shape, dtype=np.int64)
    for i in range(ndim):
        sh = [1] * ndim
        sh[i] = shape[i]
        idx = idx + (np.arange(shape[i], dtype=np.int64) * int(strides[i])).reshape(sh)
    return idx.reshape(-1)


class EmuLib:
    def __init__(self):
        self.err = b""
        self.launches = 0

    # --- bookkeeping
    def ttk_last_error(self):
        return self.err

    def ttk_version(self):
        return 1

    def ttk_launch_count(self):
        return self.launches

    # --- contractions
    @staticmethod
    def _strided(ptr, shape, strides):
        n = 1 + sum((e - 1) * st for e, st in zip(shape, strides) if e > 0)
        base = _dv(ptr, max(n, 1))
        return np.lib.stride_tricks.as_strided(base, shape=tuple(shape), strides=tuple(8 * st for st in strides))

    def ttk_einsum(self, s, eq, desc, out, alpha, beta):
        self.launches += 1
        eq = eq.decode() if isinstance(eq, bytes) else eq
        d = [int(v) for v in desc[:4096]]
        nops, pos, views, shapes = d[0] & 255, 1, [], []
        for _ in range(nops):
            ptr, nd = d[pos], d[pos + 1]
            shp, st = d[pos + 2:pos + 2 + nd], d[pos + 2 + nd:pos + 2 + 2 * nd]
            views.append(self._strided(ptr, shp, st))
            shapes.append(shp)
            pos += 2 + 2 * nd
        lhs, rhs = eq.replace(" ", "").split("->")
        ext = {}
        for idx, shp in zip(lhs.split(","), shapes):
            ext.update(zip(idx, shp))
        oshape = [ext[c] for c in rhs]
        if d[pos]:
            ost = d[pos + 2:pos + 2 + d[pos + 1]]
        else:
            ost, acc = [], 1
            for e in reversed(oshape):
                ost.insert(0, acc)
                acc *= e
        ov = self._strided(out, oshape, ost)
        res = alpha * np.einsum(eq, *views)
        if beta != 0.0:
            res = res + beta * ov
        ov[...] = res
        return 0

    def ttk_einsum_set_fused(self, on):
        return 1

    def ttk_einsum_stats(self, out):
        return 0

    def ttk_gemm_offs(self, s, A, B, C, offs, nb, M, N, K, alpha, beta):
        self.launches += 1
        o = _iv(offs, 3 * nb + 2 * M + 2 * N + 2 * K)
        a_b, a_m, a_k = o[:nb], o[nb:nb + M], o[nb + M:nb + M + K]
        p = nb + M + K
        b_b, b_k, b_n = o[p:p + nb], o[p + nb:p + nb + K], o[p + nb + K:p + nb + K + N]
        p += nb + K + N
        c_b, c_m, c_n = o[p:p + nb], o[p + nb:p + nb + M], o[p + nb + M:p + nb + M + N]
        ia = a_b[:, None, None] + a_m[None, :, None] + a_k[None, None, :]
        ib = b_b[:, None, None] + b_k[None, :, None] + b_n[None, None, :]
        ic = c_b[:, None, None] + c_m[None, :, None] + c_n[None, None, :]
        Av = _dv(A, ia.max() + 1)[ia]
        Bv = _dv(B, ib.max() + 1)[ib]
        Cm = _dv(C, ic.max() + 1)
        res = alpha * np.einsum("bmk,bkn->bmn", Av, Bv)
        if beta != 0.0:
            res = res + beta * Cm[ic]
        Cm[ic] = res
        return 0

    # --- element-wise
    def ttk_copy_nd(self, s, src, dst, nd, shape, ss, ds, alpha, beta):
        self.launches += 1
        i_s, i_d = _nd_index(nd, shape, ss), _nd_index(nd, shape, ds)
        if i_s.size == 0:
            return 0
        S = _dv(src, i_s.max() + 1)[i_s].copy()
        Dm = _dv(dst, i_d.max() + 1)
        v = alpha * S
        if beta != 0.0:
            v = v + beta * Dm[i_d]
        Dm[i_d] = v
        return 0

    def ttk_mul_nd(self, s, a, b, dst, nd, shape, sa, sb, ds, alpha, beta):
        self.launches += 1
        ia, ib, idd = _nd_index(nd, shape, sa), _nd_index(nd, shape, sb), _nd_index(nd, shape, ds)
        if ia.size == 0:
            return 0
        v = alpha * _dv(a, ia.max() + 1)[ia] * _dv(b, ib.max() + 1)[ib]
        Dm = _dv(dst, idd.max() + 1)
        if beta != 0.0:
            v = v + beta * Dm[idd]
        Dm[idd] = v
        return 0

    def ttk_scale_axis(self, s, src, dst, nd, shape, ss, ds, axis, scales):
        self.launches += 1
        i_s, i_d = _nd_index(nd, shape, ss), _nd_index(nd, shape, ds)
        if i_s.size == 0:
            return 0
        shp = [int(shape[i]) for i in range(nd)]
        coord = np.indices(shp)[axis].reshape(-1)
        sc = np.array([scales[i] for i in range(shp[axis])])
        v = _dv(src, i_s.max() + 1)[i_s] * sc[coord]
        _dv(dst, i_d.max() + 1)[i_d] = v
        return 0

    def ttk_dot_nd_dev(self, s, x, y, nd, shape, xs, ys, out):
        self.launches += 1
        ix, iy = _nd_index(nd, shape, xs), _nd_index(nd, shape, ys)
        v = 0.0 if ix.size == 0 else float(np.dot(_dv(x, ix.max() + 1)[ix], _dv(y, iy.max() + 1)[iy]))
        _dv(out, 1)[0] = v
        return 0

    def ttk_tt_join(self, s, a, b, out, ra, Ra, rb, Rb, mid, mode):
        self.launches += 1
        A = _dv(a, ra * mid * Ra).reshape(ra, mid, Ra)
        B = _dv(b, rb * mid * Rb).reshape(rb, mid, Rb)
        if mode == 0:
            o = np.zeros((ra + rb, mid, Ra + Rb))
            o[:ra, :, :Ra] = A
            o[ra:, :, Ra:] = B
        elif mode == 1:
            o = np.concatenate([A, B], axis=2)
        else:
            o = np.concatenate([A, B], axis=0)
        _dv(out, o.size)[:] = o.reshape(-1)
        return 0

    def ttk_axpby_nd(self, s, src, src2, dst, nd, shape, s1, s2, ds, alpha, beta, gamma):
        self.launches += 1
        i1, i2, idd = _nd_index(nd, shape, s1), _nd_index(nd, shape, s2), _nd_index(nd, shape, ds)
        if i1.size == 0:
            return 0
        t = gamma * _dv(src2, i2.max() + 1)[i2]
        v = alpha * _dv(src, i1.max() + 1)[i1]
        _dv(dst, idd.max() + 1)[idd] = v if beta == 0.0 else v + beta * t
        return 0

    def ttk_scale_axis_ss(self, s, src, dst, nd, shape, ss, ds, axis, sumsq, invert):
        self.launches += 1
        i_s, i_d = _nd_index(nd, shape, ss), _nd_index(nd, shape, ds)
        if i_s.size == 0:
            return 0
        shp = [int(shape[i]) for i in range(nd)]
        coord = np.indices(shp)[axis].reshape(-1)
        sc = np.maximum(np.sqrt(_dv(sumsq, shp[axis]).copy()), 1e-10)
        f = 1.0 / sc if invert else sc
        _dv(dst, i_d.max() + 1)[i_d] = _dv(src, i_s.max() + 1)[i_s] * f[coord]
        return 0

    def ttk_upload(self, s, host, dev, n):
        _dv(dev, n)[:] = _dv(host, n)
        return 0

    def ttk_normalize(self, s, x, out, nd, shape, xs):
        self.launches += 1
        ix = _nd_index(nd, shape, xs)
        if ix.size == 0:
            return 0
        v = _dv(x, ix.max() + 1)[ix].copy()
        d = float(np.dot(v, v))
        _dv(out, ix.size)[:] = (1.0 / np.sqrt(0.0 if 0.0 > d else d)) * v
        return 0

    def ttk_rayleigh_tail_sync(self, s, v, Mv, n, ev_out, r2_out):
        self.launches += 1
        a, b = _dv(v, n), _dv(Mv, n)
        ev = float(np.dot(a, b))
        b[:] = -ev * a + b
        ev_out._obj.value = ev
        r2_out._obj.value = float(np.dot(b, b))
        return 0

    def ttk_rayleigh_tail_dev(self, s, v, Mv, n, out2):
        self.launches += 1
        a, b = _dv(v, n), _dv(Mv, n)
        ev = float(np.dot(a, b))
        b[:] = -ev * a + b
        _dv(out2, 2)[:] = (ev, float(np.dot(b, b)))
        return 0

    def ttk_recip(self, s, src, dst, n):
        _dv(dst, n)[:] = 1.0 / _dv(src, n)
        return 0

    def ttk_fill(self, s, dst, n, v):
        _dv(dst, n)[:] = v
        return 0

    def ttk_add_diag(self, s, A, n, lda, v):
        a = _dv(A, (n - 1) * lda + n)
        a[np.arange(n) * lda + np.arange(n)] += v
        return 0

    def ttk_dot_nd_sync(self, s, x, y, nd, shape, xs, ys, out):
        ix, iy = _nd_index(nd, shape, xs), _nd_index(nd, shape, ys)
        val = float(np.dot(_dv(x, ix.max() + 1)[ix], _dv(y, iy.max() + 1)[iy])) if ix.size else 0.0
        out._obj.value = val
        return 0

    def ttk_einsum_batch_begin(self, s):
        return 0

    def ttk_einsum_batch_flush(self, s):
        return 0

    def ttk_einsum_batch_end(self, s):
        return 0

    def ttk_einsum_batch_stats(self, out):
        return 0

    def ttk_rank_scan_sync(self, s, res, negs, n, nq, out):
        r = _dv(res, n)
        ng = _dv(negs, n * nq).reshape(nq, n)
        o = np.ctypeslib.as_array((ctypes.c_double * int(nq)).from_address(ctypes.cast(out, ctypes.c_void_p).value))
        for q in range(nq):
            r[:] = -1.0 * ng[q] + r
            o[q] = float(np.dot(r, r))
        return 0

    def ttk_sumsq_batched(self, s, x, n, nb, bstride, out):
        xv = _dv(x, (nb - 1) * bstride + n)
        o = _dv(out, nb)
        for b in range(nb):
            seg = xv[b * bstride:b * bstride + n]
            o[b] = np.dot(seg, seg)
        return 0

    def ttk_sumsq_batched_strided(self, s, x, n, nb, bstride, inner, ostride, out):
        outer = n // inner
        xv = _dv(x, (nb - 1) * bstride + (outer - 1) * ostride + inner)
        o = _dv(out, nb)
        for b in range(nb):
            idx = b * bstride + (np.arange(outer)[:, None] * ostride + np.arange(inner)[None, :]).reshape(-1)
            seg = xv[idx]
            o[b] = np.dot(seg, seg)
        return 0

    def ttk_read_sync(self, s, src, dst, n):
        ctypes.memmove(dst, int(src), int(n) * 8)
        return 0

    # --- factorisations
    def ttk_svd_work(self, m, n):
        return 16

    def ttk_svd(self, s, A, m, n, U, S, Vt, work):
        a = _dv(A, m * n).reshape(m, n)
        u, sv, vt = np.linalg.svd(a, full_matrices=False)
        k = min(m, n)
        _dv(U, m * k)[:] = u.ravel()
        _dv(S, k)[:] = sv
        _dv(Vt, k * n)[:] = vt.ravel()
        return 0

    def ttk_qr_work(self, m, n):
        return 16

    def ttk_qr(self, s, A, m, n, Q, R, work):
        a = _dv(A, m * n).reshape(m, n)
        q, r = np.linalg.qr(a, mode="reduced")
        k = min(m, n)
        _dv(Q, m * k)[:] = q.ravel()
        _dv(R, k * n)[:] = r.ravel()
        return 0

    def ttk_cholesky_sync(self, s, A, n):
        a = _dv(A, n * n).reshape(n, n)
        try:
            L = np.linalg.cholesky(a)
        except np.linalg.LinAlgError:
            self.err = b"not positive definite"
            return 3
        a[:] = L
        return 0

    def ttk_trsm_lower(self, s, L, n, B, nrhs, ldb, trans):
        l = _dv(L, n * n).reshape(n, n)
        b = np.lib.stride_tricks.as_strided(_dv(B, (n - 1) * ldb + nrhs), shape=(n, nrhs), strides=(ldb * 8, 8))
        b[:] = sla.solve_triangular(l.T if trans else l, b.copy(), lower=not trans)
        return 0

    def ttk_lu_sync(self, s, A, n, piv, work, rcond):
        a = _dv(A, n * n).reshape(n, n)
        anorm = np.abs(a).sum(axis=0).max()
        lu, p = sla.lu_factor(a.copy(), check_finite=False)
        if np.any(np.diag(lu) == 0):
            self.err = b"singular"
            return 4
        a[:] = lu
        _i32(piv, n)[:] = p
        inv1 = np.abs(sla.lu_solve((lu, p), np.eye(n))).sum(axis=0).max()
        rcond._obj.value = 1.0 / (anorm * inv1) if anorm > 0 else 0.0
        return 0

    def ttk_lu_solve(self, s, LU, n, piv, B, nrhs, ldb):
        lu = _dv(LU, n * n).reshape(n, n)
        p = _i32(piv, n).copy()
        b = np.lib.stride_tricks.as_strided(_dv(B, (n - 1) * ldb + nrhs), shape=(n, nrhs), strides=(ldb * 8, 8))
        b[:] = sla.lu_solve((lu, p), b.copy())
        return 0

    def ttk_syev_work(self, n):
        return 16

    def ttk_syev(self, s, A, n, ev, W, work):
        a = _dv(A, n * n).reshape(n, n)
        w, v = np.linalg.eigh(a)
        _dv(ev, n)[:] = w
        _dv(W, n * n)[:] = v.ravel()
        return 0

    def ttk_contract_timing(self, on):
        return 0

    def ttk_contract_stats(self, out, reset):
        _dv(out, 5)[:] = 0.0
        return 0

    def ttk_qr_set_big_threshold(self, k):
        return 48

    def ttk_svd_tol(self, s, A, m, n, U, S, Vt, work, defl):
        return self.ttk_svd(s, A, m, n, U, S, Vt, work)

    def ttk_svd_tol_read(self, s, A, m, n, U, S, Vt, work, defl, s_host):
        rc = self.ttk_svd_tol(s, A, m, n, U, S, Vt, work, defl)
        return rc or self.ttk_read_sync(s, S, s_host, min(m, n))

    def ttk_svd_set_big_threshold(self, p):
        return 64

    def ttk_svd_set_timing(self, on):
        return 0

    def ttk_debug_counters(self, out, reset):
        return 0

    def ttk_syev_extreme_work(self, n):
        return 16

    def ttk_syev_extreme(self, s, A, n, which, ev, vec, work):
        a = _dv(A, n * n).reshape(n, n)
        w, v = np.linalg.eigh(0.5 * (a + a.T))
        j = n - 1 if which else 0
        _dv(ev, 1)[0] = w[j]
        _dv(vec, n)[:] = v[:, j]
        return 0

    # --- LGMRES (same semantics as csrc/ttk_lgmres.hip)
    @staticmethod
    def _hh(base, max_k):
        ld = max_k + 1
        tot = 2 * (max_k + 2) * ld + (max_k + 2) + 2 * ld + 8
        h = _dv(base, tot)
        HH = h[:(max_k + 2) * ld].reshape(max_k + 2, ld)
        HES = h[(max_k + 2) * ld:2 * (max_k + 2) * ld].reshape(max_k + 2, ld)
        o = 2 * (max_k + 2) * ld
        GRS = h[o:o + max_k + 2]
        CC = h[o + max_k + 2:o + max_k + 2 + ld]
        SS = h[o + max_k + 2 + ld:o + max_k + 2 + 2 * ld]
        return HH, HES, GRS, CC, SS

    def ttk_lgmres_arnoldi_sync(self, s, V, n, it, hh, max_k, haptol, res_out, flags):
        Vm = _dv(V, (it + 2) * n).reshape(it + 2, n)
        HH, HES, GRS, CC, SS = self._hh(hh, max_k)
        w = Vm[it + 1]
        h = Vm[:it + 1] @ w
        w -= h @ Vm[:it + 1]
        tt = float(np.sqrt(w @ w))
        HH[:it + 1, it] = h
        HES[:it + 1, it] = h
        HH[it + 1, it] = tt
        HES[it + 1, it] = tt
        hapbnd = min(abs(tt / GRS[it]), haptol)
        hapend = not (tt > hapbnd)
        if not hapend:
            w *= 1.0 / tt
        for j in range(1, it + 1):
            t0 = HH[j - 1, it]
            HH[j - 1, it] = CC[j - 1] * t0 + SS[j - 1] * HH[j, it]
            HH[j, it] = CC[j - 1] * HH[j, it] - SS[j - 1] * t0
        res, null = 0.0, 0
        if not hapend:
            hv, hv1 = HH[it, it], HH[it + 1, it]
            tr = np.sqrt(hv * hv + hv1 * hv1)
            if tr == 0.0:
                null = 1
            else:
                CC[it], SS[it] = hv / tr, hv1 / tr
                GRS[it + 1] = -(SS[it] * GRS[it])
                GRS[it] = CC[it] * GRS[it]
                HH[it, it] = CC[it] * hv + SS[it] * hv1
                res = abs(GRS[it + 1])
        res_out[0] = res
        res_out[1] = HH[it, it]
        flags[0] = int(hapend)
        flags[1] = null
        return 0

    def ttk_schur_build(self, ctx, ineq, m, descs, inv_I, handle):
        handle._obj.value = 0  # no native operator: the per-block path runs
        return 0

    def ttk_schur_free(self, ctx, h):
        return 0

    def ttk_lgmres_arnoldi_async(self, s, V, n, it, hh, max_k, haptol, ttol, divtol, ctl, slot, marker):
        c = _dv(ctl, 1 + 5 * (slot + 1))
        if c[0] != 0.0:
            return 0
        res, flags = (ctypes.c_double * 2)(), (ctypes.c_int * 2)()
        self.ttk_lgmres_arnoldi_sync(s, V, n, it, hh, max_k, haptol, res, flags)
        c[1 + 5 * slot:6 + 5 * slot] = (marker, res[0], flags[0], flags[1], res[1])
        r = res[0]
        if flags[0] or flags[1] or not np.isfinite(r) or r <= ttol or r >= divtol:
            c[0] = 1.0
        return 0

    def ttk_lgmres_build(self, s, hh, max_k, it, basis, nvec, n, x, aug_temp):
        HH, HES, GRS, CC, SS = self._hh(hh, max_k)
        GRS[it] = GRS[it] / HH[it, it]
        for k in range(it - 1, -1, -1):
            t0 = GRS[k]
            for j in range(k + 1, it + 1):
                t0 -= HH[k, j] * GRS[j]
            GRS[k] = t0 / HH[k, k]
        t = np.zeros(n)
        for j in range(nvec):
            t += GRS[j] * _dv(basis[j], n)
        _dv(aug_temp, n)[:] = t
        _dv(x, n)[:] += t
        return 0

    def ttk_lgmres_aug(self, s, hh, max_k, it_total, V, n, unused, aug_temp, augvec, a_augvec):
        HH, HES, GRS, CC, SS = self._hh(hh, max_k)
        avec = np.zeros(it_total + 1)
        for ii in range(it_total + 1):
            for jj in range(0, min(ii + 2, it_total + 1)):
                avec[jj] += HES[jj, ii] * GRS[ii]
        at = _dv(aug_temp, n)
        inv = 1.0 / np.sqrt(at @ at)
        _dv(augvec, n)[:] = at * inv
        Vm = _dv(V, (it_total + 1) * n).reshape(it_total + 1, n)
        _dv(a_augvec, n)[:] = (avec @ Vm) * inv
        return 0


def emulated_ttipm():
    """Import `ttipm_amd` with CPU tensors and the NumPy emulator in place of libttk.so."""
    os.environ["TTIPM_DEVICE"] = "cpu"
    os.environ["TTIPM_NO_BIND"] = "1"  # the native packer calls libttk function pointers directly
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    for k in [k for k in sys.modules if k == "ttipm_amd" or k.startswith("ttipm_amd.")]:
        del sys.modules[k]
    import ttipm_amd  # noqa: F401
    lib_mod = importlib.import_module("ttipm_amd._lib")
    lib_mod.lib = lib_mod.lib_release = EmuLib()
    for name in ("dev", "lgmres", "tt_ipm"):
        m = importlib.import_module("ttipm_amd." + name)
        m.lib = lib_mod.lib
        if hasattr(m, "lib_release"):
            m.lib_release = lib_mod.lib
    return ttipm_amd
