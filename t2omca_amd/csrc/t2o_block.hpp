// t2o_block.hpp — the attention-independent half of a transformer block
// (transformer.py:82-84 unifyheads, :130-136 residual/LN1/FFN/residual/LN2),
// forward with optional cache and backward, for one 16-row T-layout tile.
//
// With folded weights the block's attended vector is  a = Σ_h N_h z_h + b_U,
// where z_h is the head's attention-weighted average of the (original) key
// tokens.  This half maps (z, x) -> x' and is shared by the agent (per-row
// keys, observation-space attention) and the mixer (per-episode keys in LDS).
#pragma once
#include "t2o_common.hpp"

namespace t2o {

template <int E, int H, int FF>
struct PostCache {
  static constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
  f4 x[ET];    // block input (query path)
  f4 z[HET];   // per-head attention outputs
  f4 xh1[ET];
  float rs1;
  f4 f1r[FT];  // relu(W1 y + c1); the ReLU mask is f1r > 0
  f4 xh2[ET];
  float rs2;
};

// bf16: the products start from their bias (and residual) as the MFMA
// accumulator instead of adding it after, and W2's operand gets its ReLU in bf16
// (relu_bf8: packed integer max on the converted pairs, two v_pk_max_i16 per 8
// values instead of eight v_max_f32) — mixer forward step loop 2058 -> 1908
// instructions, block-1 BPTT wave 2466 -> 2247 with the paired key products.
// fp32 (the reference-precision path, 1e-5 bar) keeps its summation order.
// r2 (bf16: in = c2 + y) += W2 relu(f1)
template <int ET, int FT, bool HOIST, typename WT>
T2O_DEV void ffn_out_product(const Wts<WT>& P, int64_t off, int ld, const f4* f1, f4* r2) {
  if constexpr (sizeof(WT) == 2) {
    static_assert(FT % 2 == 0, "FFN tiles convert in pairs");
    bf4 fb[FT];
#pragma unroll
    for (int t = 0; t < FT; t += 2) {
      const bf8 v = relu_bf8(cvt8(f1[t], f1[t + 1]));
      fb[t] = lo4(v);
      fb[t + 1] = hi4(v);
    }
    matvec_b<ET, FT, HOIST, true>(P.w + off, ld, fb, r2, P.vol);
  } else {
    f4 fr[FT];
#pragma unroll
    for (int t = 0; t < FT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) fr[t][r] = fmaxf(f1[t][r], 0.f);
    matvec<ET, FT, HOIST>(P.w + off, ld, fr, r2, P.vol);  // (fp32: the caller adds c2 + y after)
  }
}

// r1 = N z + bu + x, y = LN1(r1), f1 = W1 y + c1 (bf16: bias-first accumulation)
template <int ET, int HET, int FT, bool HOIST, typename WT>
T2O_DEV void ffn_half(const Wts<WT>& P, const t2o_layout& L, int d, const f4* z, const f4* x, f4* r1, f4* y,
                      f4* xh1, float& rs1, f4* f1) {
  constexpr bool BACC = sizeof(WT) == 2;
  if constexpr (BACC) {
#pragma unroll
    for (int t = 0; t < ET; ++t) r1[t] = vec_t(P.v + L.bu[d], t) + x[t];
    matvec<ET, HET, HOIST, true>(P.w + L.N[d], HET * 16, z, r1, P.vol);
  } else {
    matvec<ET, HET, HOIST>(P.w + L.N[d], HET * 16, z, r1, P.vol);
#pragma unroll
    for (int t = 0; t < ET; ++t) r1[t] += vec_t(P.v + L.bu[d], t) + x[t];
  }
  layernorm_fwd<ET>(r1, P.v + L.g1[d], P.v + L.n1[d], y, xh1, rs1);
  if constexpr (BACC) {
#pragma unroll
    for (int t = 0; t < FT; ++t) f1[t] = vec_t(P.v + L.c1[d], t);
    matvec<FT, ET, HOIST, true>(P.w + L.W1[d], ET * 16, y, f1, P.vol);
  } else {
    matvec<FT, ET, HOIST>(P.w + L.W1[d], ET * 16, y, f1, P.vol);
#pragma unroll
    for (int t = 0; t < FT; ++t) f1[t] += vec_t(P.v + L.c1[d], t);
  }
}
// r2 = W2 relu(f1) + c2 + y
template <int ET, int FT, bool HOIST, typename WT>
T2O_DEV void ffn_tail(const Wts<WT>& P, const t2o_layout& L, int d, const f4* y, const f4* f1, f4* r2) {
  if constexpr (sizeof(WT) == 2) {
#pragma unroll
    for (int t = 0; t < ET; ++t) r2[t] = vec_t(P.v + L.c2[d], t) + y[t];
    ffn_out_product<ET, FT, HOIST>(P, L.W2[d], FT * 16, f1, r2);
  } else {
    ffn_out_product<ET, FT, HOIST>(P, L.W2[d], FT * 16, f1, r2);
#pragma unroll
    for (int t = 0; t < ET; ++t) r2[t] += vec_t(P.v + L.c2[d], t) + y[t];
  }
}

// x: in = block input, out = block output.
template <int E, int H, int FF, bool CACHE, typename WT, bool HOIST = T2O_SWZ_HOIST>
T2O_DEV void post_fwd(const Wts<WT>& P, const t2o_layout& L, int d, const f4* z, f4* x, PostCache<E, H, FF>* c) {
  constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
  f4 r1[ET], y[ET], xh1[ET], f1[FT], r2[ET];
  float rs1;
  ffn_half<ET, HET, FT, HOIST>(P, L, d, z, x, r1, y, xh1, rs1, f1);
  ffn_tail<ET, FT, HOIST>(P, L, d, y, f1, r2);
  if constexpr (CACHE) {
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      c->x[t] = x[t];
      c->xh1[t] = xh1[t];
    }
#pragma unroll
    for (int t = 0; t < HET; ++t) c->z[t] = z[t];
#pragma unroll
    for (int t = 0; t < FT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) c->f1r[t][r] = fmaxf(f1[t][r], 0.f);
    c->rs1 = rs1;
  }
  f4 xh2[ET];
  float rs2;
  layernorm_fwd<ET>(r2, P.v + L.g2[d], P.v + L.n2[d], x, xh2, rs2);
  if constexpr (CACHE) {
#pragma unroll
    for (int t = 0; t < ET; ++t) c->xh2[t] = xh2[t];
    c->rs2 = rs2;
  }
}

// gx: grad wrt block output.  Produces gz (grad wrt z, HET tiles) and gres
// (grad wrt the block input through the LN1 residual).  The operands of the
// big weight grads (N, W1, W2) and of the bu / c1 / c2 / g1 / n1 grads go to
// the wave's tape tile (TapeRec; null: no tape); the LN2 vector grads go to
// the workgroup's global slab gs (layout G).
// Weights are read from P (LDS); transposed products use matvec_t.
template <int E, int H, int FF, typename WT>
T2O_DEV void post_bwd(const Wts<WT>& P, const t2o_layout& L, const t2o_layout& G,
                      float* __restrict__ gs, WT* __restrict__ rec, int d, const PostCache<E, H, FF>& c,
                      const f4* gx, f4* gz, f4* gres, f4* ln2) {
  constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
  using R = TapeRec<E, H, FF>;
  // LN2: x' = xh2*g2 + n2 — per-lane partial sums over the wave's steps
  // (ln2[0..ET) d g2, ln2[ET..2ET) d n2), reduced once by the caller (ln2_flush)
#pragma unroll
  for (int t = 0; t < ET; ++t) {
    ln2[t] += gx[t] * c.xh2[t];
    ln2[ET + t] += gx[t];
  }
  f4 gr2[ET];
  layernorm_bwd<ET>(gx, c.xh2, c.rs2, P.v + L.g2[d], gr2);
  // r2 = W2 relu(f1) + c2 + y
  if (rec) rec_store<R::SIZE, ET>(rec, R::GR2, gr2);
  f4 gf1[FT];
  matvec_tr<FT, ET>(P, L.W2[d], FF, L.W2T[d], E, gr2, gf1);
#pragma unroll
  for (int t = 0; t < FT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) gf1[t][r] = c.f1r[t][r] > 0.f ? gf1[t][r] : 0.f;
  f4 gy[ET];
  matvec_tr<ET, FT>(P, L.W1[d], E, L.W1T[d], FF, gf1, gy);
#pragma unroll
  for (int t = 0; t < ET; ++t) gy[t] += gr2[t];
  // LN1: y = xh1*g1 + n1 (y, f1, gf1 and the g1 / n1 grads come from the tape's
  // (x̂1, gr2): TapeRec)
  if (rec) rec_store<R::SIZE, ET>(rec, R::XH1, c.xh1);
  layernorm_bwd<ET>(gy, c.xh1, c.rs1, P.v + L.g1[d], gres);
  // r1 = N z + b_U + x
  if (rec) {
    rec_store<R::SIZE, ET>(rec, R::GRES, gres);
    rec_store<R::SIZE, HET>(rec, R::Z, c.z);
  }
  matvec_tr<HET, ET>(P, L.N[d], H * E, L.NT[d], E, gres, gz);
}

// Lean variant for the two-wave pipelined kernels, whose cache must live in
// half a register file: the tape operands already known in the forward (x, z)
// are written to the record by the recompute itself, and the FFN's ReLU is
// kept as a bit mask (its only use in the backward).  Same records, same math.
template <int E, int H, int FF>
struct PostCacheLean {
  static constexpr int ET = E / 16, FT = FF / 16;
  static_assert(FT * 4 <= 32, "ReLU mask is one 32-bit register");
  f4 xh1[ET];
  float rs1;
  uint32_t relu;  // bit 4t + r: f1[t][r] > 0
  f4 xh2[ET];
  float rs2;
};

// R: the tape record (TapeRec; TapeRecA has no X / Z fields — its writer keeps
// dN's operands itself).
template <int E, int H, int FF, typename WT, typename R = TapeRec<E, H, FF>, int CP = 0>
T2O_DEV void post_fwd_lean(const Wts<WT>& P, const t2o_layout& L, int d, const f4* z, f4* x,
                           PostCacheLean<E, H, FF>* c, const MaskedRec<WT, CP>& rec) {
  constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
  if constexpr (R::X >= 0) rec.template store<ET>(R::X, x);
  if constexpr (R::Z >= 0) rec.template store<HET>(R::Z, z);
  f4 r1[ET], y[ET], f1[FT], r2[ET];
  ffn_half<ET, HET, FT, T2O_SWZ_HOIST>(P, L, d, z, x, r1, y, c->xh1, c->rs1, f1);
  uint32_t m = 0;
#pragma unroll
  for (int t = 0; t < FT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) m |= (f1[t][r] > 0.f ? 1u : 0u) << (4 * t + r);
  c->relu = m;
  ffn_tail<ET, FT, T2O_SWZ_HOIST>(P, L, d, y, f1, r2);
  layernorm_fwd<ET>(r2, P.v + L.g2[d], P.v + L.n2[d], x, c->xh2, c->rs2);
}

// post_bwd for the lean cache (the X, Z record fields were written forward)
template <int E, int H, int FF, typename WT, typename R = TapeRec<E, H, FF>, int CP = 0>
T2O_DEV void post_bwd_lean(const Wts<WT>& P, const t2o_layout& L, float* __restrict__ gs, const MaskedRec<WT, CP>& rec,
                           int d, const PostCacheLean<E, H, FF>& c, const f4* gx, f4* gz, f4* gres, f4* ln2) {
  constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
#pragma unroll
  for (int t = 0; t < ET; ++t) {
    ln2[t] += gx[t] * c.xh2[t];
    ln2[ET + t] += gx[t];
  }
  f4 gr2[ET];
  layernorm_bwd<ET>(gx, c.xh2, c.rs2, P.v + L.g2[d], gr2);
  rec.template store<ET>(R::GR2, gr2);
  f4 gf1[FT];
  matvec_tr<FT, ET>(P, L.W2[d], FF, L.W2T[d], E, gr2, gf1);
#pragma unroll
  for (int t = 0; t < FT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)  // bit 4t + r of the mask as 0 / -1 (v_bfe_i32), ANDed onto the grad
      gf1[t][r] = __int_as_float(__float_as_int(gf1[t][r]) & __builtin_amdgcn_sbfe((int)c.relu, 4 * t + r, 1));
  f4 gy[ET];
  matvec_tr<ET, FT>(P, L.W1[d], E, L.W1T[d], FF, gf1, gy);
#pragma unroll
  for (int t = 0; t < ET; ++t) gy[t] += gr2[t];
  rec.template store<ET>(R::XH1, c.xh1);
  layernorm_bwd<ET>(gy, c.xh1, c.rs1, P.v + L.g1[d], gres);
  rec.template store<ET>(R::GRES, gres);
  matvec_tr<HET, ET>(P, L.N[d], H * E, L.NT[d], E, gres, gz);
  (void)gs;
}

// Layout whose block-0 slots hold block d's offsets: the block code is then
// called with the constant d = 0, and every offset it reads is a scalar.  L is
// the kernel-argument layout (or a compile-time one indexed by a constant d): a
// run-time d indexes the kernel-argument fields directly, one scalar load each.
// (Round 3 replaced the indexing by a select over the T2O_MAX_DEPTH entries of
// every field, for a compile-time layout indexed at run time; on the kernel-
// argument layout that kept 4x the offsets live in SGPRs and cost the agent
// BPTT 0.543 -> 0.604 ms, bisected in profiles/r4_bisect/.)
T2O_DEV t2o_layout block_view(const t2o_layout& L, int d) {
  t2o_layout V = L;
  V.M[0] = L.M[d];
  V.MT[0] = L.MT[d];
  V.N[0] = L.N[d];
  V.NT[0] = L.NT[d];
  V.bu[0] = L.bu[d];
  V.g1[0] = L.g1[d];
  V.n1[0] = L.n1[d];
  V.W1[0] = L.W1[d];
  V.W1T[0] = L.W1T[d];
  V.c1[0] = L.c1[d];
  V.W2[0] = L.W2[d];
  V.W2T[0] = L.W2T[d];
  V.c2[0] = L.c2[d];
  V.g2[0] = L.g2[d];
  V.n2[0] = L.n2[d];
  return V;
}

// LN2 vector grads of every block, summed over this wave's rows and steps
template <int E, int D>
T2O_DEV void ln2_flush(float* __restrict__ gs, const t2o_layout& G, const f4 (&ln2)[D][2 * (E / 16)]) {
  constexpr int ET = E / 16;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    vec_accumulate_g<ET>(gs + G.g2[d], &ln2[d][0]);
    vec_accumulate_g<ET>(gs + G.n2[d], &ln2[d][ET]);
  }
}

}  // namespace t2o
