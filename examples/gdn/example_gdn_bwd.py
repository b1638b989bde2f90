"""Gated DeltaNet chunked backward on tilelang kernels (reference: examples/gdn/
example_chunk_o_bwd.py, example_chunk_delta_bwd.py, example_wy_fast_bwd_split.py; FLA's
chunk_gated_delta_rule_bwd).  Forward and notation: example_gdn.py.

Per chunk c (C rows, g = within-chunk cumulative log-gate, G_c = g of the last row,
Gam[s, t] = exp(g_s - g_t), M = causal mask) the forward is

    A = strict_tril(beta_s (k_s . k_t) Gam),  Tm = (I + A)^-1
    w = Tm (beta e^g k),  u = Tm (beta v)
    v_new = u - w h_c,    h_{c+1} = e^{G_c} h_c + (k e^{G_c - g})^T v_new
    o = scale [e^g q h_c + (q k^T * Gam * M) v_new]

and the backward runs as four kernels (dH_{c+1} = dL/dh_{c+1}):

  chunk_bwd_dv_local   dv_loc = scale (q k^T * Gam * M)^T do                        per chunk
  chunk_delta_bwd      reverse over chunks, state dH in fp32 registers:             sequential
                         dv_tot = dv_loc + (k e^{G_c - g}) dH_{c+1}
                         dH_c   = e^{G_c} dH_{c+1} + scale (e^g q)^T do - w^T dv_tot
  chunk_bwd_dqkwg      dA = do v_new^T;  dq = scale (e^g (do h_c^T) + (dA Gam M) k)   per chunk
                         dk = scale (dA Gam M)^T q + e^{G_c - g} (v_new dH^T);  dw = -dv_tot h_c^T
                         dg: row/column sums of the gate products (exp'(x) = exp(x))
  wy_fast_bwd          dXw = Tm^T dw, dXu = Tm^T du, dA = -Tm^T (dw Xw^T + du Xu^T) Tm^T,   per chunk
                         dk += beta e^g dXw + (dA beta Gam) k + (dA beta Gam)^T k;  dv = beta dXu
                         dbeta, dg, then dg -> d(raw g) by a reverse within-chunk cumsum

Every product is an MFMA tile GEMM on bf16 LDS operands with fp32 accumulation (the precision
FLA uses); gate factors are applied in fp32.  One workgroup per (chunk, batch*head) except the
sequential dH walk (one per (batch*head, DV slice), like the forward's chunk_delta_h).
"""
import argparse
import functools

import tilelang
import tilelang.language as T

from example_gdn import FAST_MATH, LOG2E, chunk_cumsum, chunk_scaled_dot_kkt, solve_tril, wy_fast, chunk_delta_h


def _ex(x):
    return T.exp2(x * LOG2E)


@tilelang.jit(out_idx=[4], pass_configs=FAST_MATH)
def chunk_bwd_dv_local(B, S, H, DK, DV, C=64, scale=None, threads=256, dtype="bfloat16"):
    scale = DK**-0.5 if scale is None else scale

    @T.prim_func
    def main(Q: T.Tensor([B, S, H, DK], dtype), K: T.Tensor([B, S, H, DK], dtype), Gc: T.Tensor([B, S, H], "float32"),
             dO: T.Tensor([B, S, H, DV], dtype), dV: T.Tensor([B, S, H, DV], dtype)):
        with T.Kernel(S // C, B * H, threads=threads) as (bc, bbh):
            b, h = bbh // H, bbh % H
            q_s = T.alloc_shared([C, DK], dtype)
            k_s = T.alloc_shared([C, DK], dtype)
            do_s = T.alloc_shared([C, DV], dtype)
            g_s = T.alloc_shared([C], "float32")
            kq = T.alloc_fragment([C, C], "float32")
            pt_s = T.alloc_shared([C, C], dtype)
            dv = T.alloc_fragment([C, DV], "float32")
            T.copy(Q[b, bc * C:(bc + 1) * C, h, :], q_s)
            T.copy(K[b, bc * C:(bc + 1) * C, h, :], k_s)
            T.copy(dO[b, bc * C:(bc + 1) * C, h, :], do_s)
            T.copy(Gc[b, bc * C:(bc + 1) * C, h], g_s)
            T.clear(kq)
            T.gemm(k_s, q_s, kq, transpose_B=True)  # [t, s] = k_t . q_s
            for t, s in T.Parallel(C, C):
                pt_s[t, s] = T.if_then_else(s >= t, kq[t, s] * _ex(g_s[s] - g_s[t]) * scale, 0.0)
            T.clear(dv)
            T.gemm(pt_s, do_s, dv)
            T.copy(dv, dV[b, bc * C:(bc + 1) * C, h, :])

    return main


@tilelang.jit(out_idx=[7, 8, 9], pass_configs=FAST_MATH)
def chunk_delta_bwd(B, S, H, DK, DV, C=64, block_DV=32, scale=None, threads=256, dtype="bfloat16"):
    """Reverse walk: Dh[c] = dL/dh_{c+1}, dv_tot, dh0 = dL/dh_0 (dht = dL/d final state)."""
    NT = S // C
    scale = DK**-0.5 if scale is None else scale

    @T.prim_func
    def main(Q: T.Tensor([B, S, H, DK], dtype), K: T.Tensor([B, S, H, DK], dtype), W: T.Tensor([B, S, H, DK], dtype),
             Gc: T.Tensor([B, S, H], "float32"), dO: T.Tensor([B, S, H, DV], dtype),
             dVloc: T.Tensor([B, S, H, DV], dtype), dHt: T.Tensor([B, H, DK, DV], "float32"),
             Dh: T.Tensor([B, NT, H, DK, DV], dtype), dVtot: T.Tensor([B, S, H, DV], dtype),
             dH0: T.Tensor([B, H, DK, DV], "float32")):
        with T.Kernel(DV // block_DV, B * H, threads=threads) as (bv, bbh):
            b, h = bbh // H, bbh % H
            dh = T.alloc_fragment([DK, block_DV], "float32")
            dh_s = T.alloc_shared([DK, block_DV], dtype)
            qg_s = T.alloc_shared([C, DK], dtype)
            kg_s = T.alloc_shared([C, DK], dtype)
            w_s = T.alloc_shared([C, DK], dtype)
            do_s = T.alloc_shared([C, block_DV], dtype)
            dvn_s = T.alloc_shared([C, block_DV], dtype)
            g_s = T.alloc_shared([C], "float32")
            dvt = T.alloc_fragment([C, block_DV], "float32")
            T.copy(dHt[b, h, :, bv * block_DV:(bv + 1) * block_DV], dh)
            for r in T.serial(NT):
                c = NT - 1 - r
                T.copy(Gc[b, c * C:(c + 1) * C, h], g_s)
                for s, d in T.Parallel(C, DK):
                    qg_s[s, d] = Q[b, c * C + s, h, d] * (_ex(g_s[s]) * scale)
                    kg_s[s, d] = K[b, c * C + s, h, d] * _ex(g_s[C - 1] - g_s[s])
                T.copy(W[b, c * C:(c + 1) * C, h, :], w_s)
                T.copy(dO[b, c * C:(c + 1) * C, h, bv * block_DV:(bv + 1) * block_DV], do_s)
                T.copy(dh, dh_s)
                T.copy(dh_s, Dh[b, c, h, :, bv * block_DV:(bv + 1) * block_DV])
                T.copy(dVloc[b, c * C:(c + 1) * C, h, bv * block_DV:(bv + 1) * block_DV], dvt)
                T.gemm(kg_s, dh_s, dvt)
                T.copy(dvt, dVtot[b, c * C:(c + 1) * C, h, bv * block_DV:(bv + 1) * block_DV])
                for s, v in T.Parallel(C, block_DV):
                    dvn_s[s, v] = -dvt[s, v]
                for d, v in T.Parallel(DK, block_DV):
                    dh[d, v] *= _ex(g_s[C - 1])
                T.gemm(qg_s, do_s, dh, transpose_A=True)
                T.gemm(w_s, dvn_s, dh, transpose_A=True)
            T.copy(dh, dH0[b, h, :, bv * block_DV:(bv + 1) * block_DV])

    return main


@tilelang.jit(out_idx=[8, 9, 10, 11], pass_configs=FAST_MATH)
def chunk_bwd_dqkwg(B, S, H, DK, DV, C=64, scale=None, threads=256, dtype="bfloat16"):
    """dq, dk (chunk_o + state parts), dw (bf16) and dg (w.r.t. the cumsummed gate, fp32)."""
    NT = S // C
    scale = DK**-0.5 if scale is None else scale

    @T.prim_func
    def main(Q: T.Tensor([B, S, H, DK], dtype), K: T.Tensor([B, S, H, DK], dtype),
             Vnew: T.Tensor([B, S, H, DV], dtype), Hs: T.Tensor([B, NT, H, DK, DV], dtype),
             Gc: T.Tensor([B, S, H], "float32"), dO: T.Tensor([B, S, H, DV], dtype),
             Dh: T.Tensor([B, NT, H, DK, DV], dtype), dVtot: T.Tensor([B, S, H, DV], dtype),
             dQ: T.Tensor([B, S, H, DK], "float32"), dK: T.Tensor([B, S, H, DK], "float32"),
             dW: T.Tensor([B, S, H, DK], dtype), dG: T.Tensor([B, S, H], "float32")):
        with T.Kernel(NT, B * H, threads=threads) as (bc, bbh):
            b, h = bbh // H, bbh % H
            q_s = T.alloc_shared([C, DK], dtype)
            k_s = T.alloc_shared([C, DK], dtype)
            do_s = T.alloc_shared([C, DV], dtype)
            vn_s = T.alloc_shared([C, DV], dtype)
            dvt_s = T.alloc_shared([C, DV], dtype)
            h_s = T.alloc_shared([DK, DV], dtype)
            dh_s = T.alloc_shared([DK, DV], dtype)
            g_s = T.alloc_shared([C], "float32")
            ds_s = T.alloc_shared([C, C], dtype)
            p_s = T.alloc_shared([C, C], "float32")
            dA = T.alloc_fragment([C, C], "float32")
            qk = T.alloc_fragment([C, C], "float32")
            dq = T.alloc_fragment([C, DK], "float32")
            dki = T.alloc_fragment([C, DK], "float32")
            dk = T.alloc_fragment([C, DK], "float32")
            dw = T.alloc_fragment([C, DK], "float32")
            hdh = T.alloc_fragment([DK, DV], "float32")
            tmp = T.alloc_fragment([C, DK], "float32")
            row = T.alloc_fragment([C], "float32")
            row2 = T.alloc_fragment([C], "float32")
            hsum = T.alloc_fragment([DK], "float32")
            dg_s = T.alloc_shared([C], "float32")
            gl = T.alloc_shared([2], "float32")
            hs_s = T.alloc_shared([DK], "float32")
            r2_s = T.alloc_shared([C], "float32")

            T.copy(Q[b, bc * C:(bc + 1) * C, h, :], q_s)
            T.copy(K[b, bc * C:(bc + 1) * C, h, :], k_s)
            T.copy(dO[b, bc * C:(bc + 1) * C, h, :], do_s)
            T.copy(Vnew[b, bc * C:(bc + 1) * C, h, :], vn_s)
            T.copy(dVtot[b, bc * C:(bc + 1) * C, h, :], dvt_s)
            T.copy(Hs[b, bc, h, :, :], h_s)
            T.copy(Dh[b, bc, h, :, :], dh_s)
            T.copy(Gc[b, bc * C:(bc + 1) * C, h], g_s)
            # dG_c gets e^{G_c} sum(h_c * dH_{c+1})
            for d, v in T.Parallel(DK, DV):
                hdh[d, v] = h_s[d, v] * dh_s[d, v]
            T.reduce_sum(hdh, hsum, dim=1)
            # products with the state
            T.clear(dA)
            T.gemm(do_s, vn_s, dA, transpose_B=True)
            T.clear(dq)
            T.gemm(do_s, h_s, dq, transpose_B=True)
            T.clear(dki)
            T.gemm(vn_s, dh_s, dki, transpose_B=True)
            T.clear(dw)
            T.gemm(dvt_s, h_s, dw, transpose_B=True)
            for s, d in T.Parallel(C, DK):
                dw[s, d] = -dw[s, d]
            T.copy(dw, dW[b, bc * C:(bc + 1) * C, h, :])
            # intra-chunk gate products: P = scale dA Gam M (as GEMM operand) and P * (q k^T) for dg
            T.clear(qk)
            T.gemm(q_s, k_s, qk, transpose_B=True)
            for s, t in T.Parallel(C, C):
                dA[s, t] = T.if_then_else(t <= s, dA[s, t] * _ex(g_s[s] - g_s[t]) * scale, 0.0)
            T.copy(dA, ds_s)
            for s, t in T.Parallel(C, C):
                p_s[s, t] = dA[s, t] * qk[s, t]
            # dq = scale e^g (do h^T) + P k
            for s, d in T.Parallel(C, DK):
                dq[s, d] = dq[s, d] * (_ex(g_s[s]) * scale)
            for s, d in T.Parallel(C, DK):
                tmp[s, d] = dq[s, d] * q_s[s, d]
            T.reduce_sum(tmp, row, dim=1)  # inter part of dg
            T.gemm(ds_s, k_s, dq)
            T.copy(dq, dQ[b, bc * C:(bc + 1) * C, h, :])
            # dk = P^T q + e^{G_c - g} (v_new dH^T)
            for s, d in T.Parallel(C, DK):
                dki[s, d] = dki[s, d] * _ex(g_s[C - 1] - g_s[s])
            for s, d in T.Parallel(C, DK):
                tmp[s, d] = dki[s, d] * k_s[s, d]
            T.reduce_sum(tmp, row2, dim=1)
            T.clear(dk)
            T.gemm(ds_s, q_s, dk, transpose_A=True)
            for s, d in T.Parallel(C, DK):
                dk[s, d] = dk[s, d] + dki[s, d]
            T.copy(dk, dK[b, bc * C:(bc + 1) * C, h, :])
            # dg_s = inter + rowsum(P*qk) - colsum(P*qk) - e^{G_c-g_s} k_s.(v_new dH^T)_s ; last row += ...
            for s in T.Parallel(C):
                dg_s[s] = row[s] - row2[s]
            for s in T.Parallel(C):
                acc_r = T.alloc_var("float32")
                acc_c = T.alloc_var("float32")
                acc_r = 0.0
                acc_c = 0.0
                for t in T.serial(C):
                    acc_r = acc_r + p_s[s, t]
                    acc_c = acc_c + p_s[t, s]
                dg_s[s] = dg_s[s] + acc_r - acc_c
            T.copy(hsum, hs_s)
            T.copy(row2, r2_s)
            for s in T.Parallel(1):
                tot = T.alloc_var("float32")
                tot2 = T.alloc_var("float32")
                tot = 0.0
                tot2 = 0.0
                for d in T.serial(DK):
                    tot = tot + hs_s[d]
                for t in T.serial(C):
                    tot2 = tot2 + r2_s[t]
                gl[0] = tot * _ex(g_s[C - 1])
                gl[1] = tot2
            for s in T.Parallel(C):
                dG[b, bc * C + s, h] = dg_s[s] + T.if_then_else(s == C - 1, gl[0] + gl[1], 0.0)

    return main


@tilelang.jit(out_idx=[9, 10, 11, 12], pass_configs=FAST_MATH)
def wy_fast_bwd(B, S, H, DK, DV, C=64, threads=256, dtype="bfloat16"):
    """WY-representation backward + the gate cumsum backward.  dK_in / dG_in (from
    chunk_bwd_dqkwg) are added, so the outputs are the final dk, dv, dbeta, dg (w.r.t. raw g)."""

    @T.prim_func
    def main(K: T.Tensor([B, S, H, DK], dtype), V: T.Tensor([B, S, H, DV], dtype), Beta: T.Tensor([B, S, H], "float32"),
             Gc: T.Tensor([B, S, H], "float32"), Tm: T.Tensor([B, S, H, C], "float32"),
             dW: T.Tensor([B, S, H, DK], dtype), dU: T.Tensor([B, S, H, DV], dtype),
             dK_in: T.Tensor([B, S, H, DK], "float32"), dG_in: T.Tensor([B, S, H], "float32"),
             dK: T.Tensor([B, S, H, DK], "float32"), dV: T.Tensor([B, S, H, DV], "float32"),
             dBeta: T.Tensor([B, S, H], "float32"), dG: T.Tensor([B, S, H], "float32")):
        with T.Kernel(S // C, B * H, threads=threads) as (bc, bbh):
            b, h = bbh // H, bbh % H
            k_s = T.alloc_shared([C, DK], dtype)
            xw_s = T.alloc_shared([C, DK], dtype)
            xu_s = T.alloc_shared([C, DV], dtype)
            dw_s = T.alloc_shared([C, DK], dtype)
            du_s = T.alloc_shared([C, DV], dtype)
            tm_s = T.alloc_shared([C, C], dtype)
            m_s = T.alloc_shared([C, C], dtype)
            ca_s = T.alloc_shared([C, C], dtype)
            dA_f = T.alloc_shared([C, C], "float32")
            kk_f = T.alloc_shared([C, C], "float32")
            g_s = T.alloc_shared([C], "float32")
            be_s = T.alloc_shared([C], "float32")
            dg_s = T.alloc_shared([C], "float32")
            dxw = T.alloc_fragment([C, DK], "float32")
            dxu = T.alloc_fragment([C, DV], "float32")
            dtm = T.alloc_fragment([C, C], "float32")
            mm = T.alloc_fragment([C, C], "float32")
            kk = T.alloc_fragment([C, C], "float32")
            dk = T.alloc_fragment([C, DK], "float32")
            tmpk = T.alloc_fragment([C, DK], "float32")
            tmpv = T.alloc_fragment([C, DV], "float32")
            r1 = T.alloc_fragment([C], "float32")
            r2 = T.alloc_fragment([C], "float32")

            T.copy(Gc[b, bc * C:(bc + 1) * C, h], g_s)
            T.copy(Beta[b, bc * C:(bc + 1) * C, h], be_s)
            T.copy(K[b, bc * C:(bc + 1) * C, h, :], k_s)
            for s, d in T.Parallel(C, DK):
                xw_s[s, d] = K[b, bc * C + s, h, d] * (be_s[s] * _ex(g_s[s]))
            for s, d in T.Parallel(C, DV):
                xu_s[s, d] = V[b, bc * C + s, h, d] * be_s[s]
            for s, t in T.Parallel(C, C):
                tm_s[s, t] = Tm[b, bc * C + s, h, t]
            T.copy(dW[b, bc * C:(bc + 1) * C, h, :], dw_s)
            T.copy(dU[b, bc * C:(bc + 1) * C, h, :], du_s)
            # dX = Tm^T dY
            T.clear(dxw)
            T.gemm(tm_s, dw_s, dxw, transpose_A=True)
            T.clear(dxu)
            T.gemm(tm_s, du_s, dxu, transpose_A=True)
            # dTm = dw Xw^T + du Xu^T ;  dA = -(Tm^T dTm) Tm^T, strictly lower
            T.clear(dtm)
            T.gemm(dw_s, xw_s, dtm, transpose_B=True)
            T.gemm(du_s, xu_s, dtm, transpose_B=True)
            T.copy(dtm, m_s)
            T.clear(mm)
            T.gemm(tm_s, m_s, mm, transpose_A=True)
            T.copy(mm, m_s)
            T.clear(dtm)
            T.gemm(m_s, tm_s, dtm, transpose_B=True)
            T.clear(kk)
            T.gemm(k_s, k_s, kk, transpose_B=True)
            for s, t in T.Parallel(C, C):
                dA_f[s, t] = T.if_then_else(t < s, -dtm[s, t], 0.0)
                kk_f[s, t] = kk[s, t]
            # coefficient of k_s k_t in A: dA beta_s Gam
            for s, t in T.Parallel(C, C):
                ca_s[s, t] = dA_f[s, t] * be_s[s] * _ex(g_s[s] - g_s[t])
            T.copy(dK_in[b, bc * C:(bc + 1) * C, h, :], dk)
            for s, d in T.Parallel(C, DK):
                dk[s, d] = dk[s, d] + dxw[s, d] * (be_s[s] * _ex(g_s[s]))
            T.gemm(ca_s, k_s, dk)
            T.gemm(ca_s, k_s, dk, transpose_A=True)
            T.copy(dk, dK[b, bc * C:(bc + 1) * C, h, :])
            for s, d in T.Parallel(C, DV):
                tmpv[s, d] = dxu[s, d] * be_s[s]
            T.copy(tmpv, dV[b, bc * C:(bc + 1) * C, h, :])
            # dbeta, dg rows
            for s, d in T.Parallel(C, DK):
                tmpk[s, d] = dxw[s, d] * k_s[s, d]
            T.reduce_sum(tmpk, r1, dim=1)  # k . dXw
            for s, d in T.Parallel(C, DV):
                tmpv[s, d] = dxu[s, d] * V[b, bc * C + s, h, d]
            T.reduce_sum(tmpv, r2, dim=1)  # v . dXu
            for s in T.Parallel(C):
                ab = T.alloc_var("float32")
                ar = T.alloc_var("float32")
                ac = T.alloc_var("float32")
                ab = 0.0
                ar = 0.0
                ac = 0.0
                for t in T.serial(C):
                    gam = _ex(g_s[s] - g_s[t])
                    ab = ab + dA_f[s, t] * kk_f[s, t] * gam
                    ar = ar + dA_f[s, t] * kk_f[s, t] * gam * be_s[s]
                    ac = ac + dA_f[t, s] * kk_f[t, s] * _ex(g_s[t] - g_s[s]) * be_s[t]
                eg = _ex(g_s[s])
                dBeta[b, bc * C + s, h] = eg * r1[s] + r2[s] + ab
                dg_s[s] = dG_in[b, bc * C + s, h] + be_s[s] * eg * r1[s] + ar - ac
            # g was a within-chunk inclusive cumsum: d(raw g_s) = sum_{s' >= s} dg_{s'}
            for s in T.Parallel(C):
                acc = T.alloc_var("float32")
                acc = 0.0
                for t in T.serial(C):
                    acc = acc + T.if_then_else(t >= s, dg_s[t], 0.0)
                dG[b, bc * C + s, h] = acc

    return main


@functools.lru_cache(maxsize=None)
def _bwd_kernels(B, S, H, DK, DV, C, block_DV, tgt):

    def k_(impl, *args, out_idx):
        return tilelang.compile(impl.get_tir(*args), out_idx=out_idx, target=tgt)

    return dict(cum=k_(chunk_cumsum, B, S, H, C, out_idx=[1]),
                kkt=k_(chunk_scaled_dot_kkt, B, S, H, DK, C, out_idx=[3]),
                tril=k_(solve_tril, B, S, H, C, out_idx=[1]), wy=k_(wy_fast, B, S, H, DK, DV, C, out_idx=[5, 6]),
                h=k_(chunk_delta_h, B, S, H, DK, DV, C, min(block_DV, DV), out_idx=[4, 5, 6]),
                dvl=k_(chunk_bwd_dv_local, B, S, H, DK, DV, C, out_idx=[4]),
                dhu=k_(chunk_delta_bwd, B, S, H, DK, DV, C, min(block_DV, DV), out_idx=[7, 8, 9]),
                dqkwg=k_(chunk_bwd_dqkwg, B, S, H, DK, DV, C, out_idx=[8, 9, 10, 11]),
                wyb=k_(wy_fast_bwd, B, S, H, DK, DV, C, out_idx=[9, 10, 11, 12]))


def chunk_gated_delta_rule_bwd(q, k, v, g, beta, do, dht=None, C=64, block_DV=32, target=None):
    """Gradients (dq, dk, dv, dg, dbeta, dh0) of the chunked GDN forward (fp32, scale = DK^-0.5).
    The forward intermediates (cumsummed gate, Tm, w, u, h_c, v_new) are recomputed, as FLA does."""
    import torch
    B, S, H, DK = q.shape
    DV = v.shape[-1]
    tgt = target or ("cpu" if q.device.type == "cpu" else "hip")
    ks = _bwd_kernels(B, S, H, DK, DV, C, block_DV, tgt)
    beta = beta.float().contiguous()
    gc = ks["cum"](g.float().contiguous())
    Tm = ks["tril"](ks["kkt"](k, beta, gc))
    w, u = ks["wy"](k, v, beta, gc, Tm)
    hs, vnew, _ = ks["h"](k, w, u, gc)
    do = do.to(q.dtype).contiguous()
    dht = torch.zeros(B, H, DK, DV, device=q.device) if dht is None else dht.float().contiguous()
    dv_loc = ks["dvl"](q, k, gc, do)
    dh, dv_tot, dh0 = ks["dhu"](q, k, w, gc, do, dv_loc, dht)
    dq, dk1, dw, dg1 = ks["dqkwg"](q, k, vnew, hs, gc, do, dh, dv_tot)
    dk, dv, dbeta, dg = ks["wyb"](k, v, beta, gc, Tm, dw, dv_tot, dk1, dg1)
    return dq, dk, dv, dg, dbeta, dh0


class ChunkGatedDeltaRule:
    """``ChunkGatedDeltaRule.apply(q, k, v, g, beta)`` -> o: autograd over the tilelang forward and
    backward kernels (final-state output not differentiated here)."""

    @staticmethod
    def apply(q, k, v, g, beta):
        import torch
        from example_gdn import chunk_gated_delta_rule

        class _Fn(torch.autograd.Function):

            @staticmethod
            def forward(ctx, q, k, v, g, beta):
                o, _ = chunk_gated_delta_rule(q, k, v, g, beta)
                ctx.save_for_backward(q, k, v, g, beta)
                return o

            @staticmethod
            def backward(ctx, do):
                q, k, v, g, beta = ctx.saved_tensors
                dq, dk, dv, dg, dbeta, _ = chunk_gated_delta_rule_bwd(q, k, v, g, beta, do)
                return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), dg.to(g.dtype), dbeta.to(beta.dtype)

        return _Fn.apply(q, k, v, g, beta)


def reference_grads(q, k, v, g, beta, do):
    """fp32 autograd through the token recurrence (example_gdn.naive_recurrent)."""
    import torch
    from example_gdn import naive_recurrent
    xs = [x.detach().float().cpu().requires_grad_(True) for x in (q, k, v, g, beta)]
    o, _ = naive_recurrent(*xs)
    o.backward(do.float().cpu())
    return [x.grad for x in xs]


def main(B=1, S=8192, H=16, DK=128, DV=128):
    import torch
    from example_gdn import make_inputs
    q, k, v, g, beta = make_inputs(1, 256, 2, DK, DV, "cuda")
    do = torch.randn(1, 256, 2, DV, device="cuda", dtype=torch.bfloat16)
    got = chunk_gated_delta_rule_bwd(q, k, v, g, beta, do)[:5]
    ref = reference_grads(q, k, v, g, beta, do)
    for n, a, r in zip(("dq", "dk", "dv", "dg", "dbeta"), got, ref):
        err = (a.float().cpu() - r).abs().max().item() / max(1.0, r.abs().max().item())
        print(f"{n}: rel max err {err:.3e}")
    q, k, v, g, beta = make_inputs(B, S, H, DK, DV, "cuda")
    do = torch.randn(B, S, H, DV, device="cuda", dtype=torch.bfloat16)
    from tilelang.profiler import do_bench
    chunk_gated_delta_rule_bwd(q, k, v, g, beta, do)
    lat = do_bench(lambda: chunk_gated_delta_rule_bwd(q, k, v, g, beta, do))
    print(f"GDN chunked bwd B{B} S{S} H{H} K{DK} V{DV}: {lat:.3f} ms (forward recompute + 4 bwd kernels)")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--seq", type=int, default=8192)
    p.add_argument("--heads", type=int, default=16)
    a = p.parse_args()
    main(S=a.seq, H=a.heads)
