// t2o_agent_block.hpp — one transformer block of the agent for a 16-row tile,
// forward (optionally caching what the backward needs) and backward.
//
// Reference: transformer.py:40-140 called from transf_agent.py:54-76.  Only
// query row 0 (the hidden token) is propagated: every block attends over the
// ORIGINAL tokens [h, We·o_1+b_e, ..., We·o_n+b_e] (transformer.py:140 returns
// the unchanged keys) and Q is read from token 0 (transf_agent.py:71), so the
// other query rows never influence the output.
//
// Per row, with folded weights (t2o_pack.hip):
//   u_h = M_h x;  w_h = We_ᵀ u_h (F-dim);  c_h = u_h·b_e
//   s_h0 = u_h·h;  s_hj = w_h·o_j + c_h;  p_h = softmax(s_h)
//   ô_h = Σ_j p_hj o_j;  P_h = Σ_j p_hj;  z_h = p_h0 h + We ô_h + P_h b_e
// then the shared post-attention half (t2o_block.hpp).  Observation features
// live in the T-layout over a 16-padded F axis: lane group g holds
// o_j[4g .. 4g+3], so every per-entity dot product is a packed multiply-add pair
// plus a 4-lane reduction, and no entity embedding is ever materialised.  The
// reduction scatters (rsum4_n): lane group g ends with entity 4i + g's score, the
// softmax runs on ceil(NE/4) values per lane, and only the probabilities are
// broadcast back (bcast4_n) for ô — the same per-row math with a quarter of the
// softmax VALU (16 entities: agent forward step loop 3608 -> 3067 instructions).
#pragma once
#include "t2o_block.hpp"

namespace t2o {

// Entity batches of the softmax: after the score reduction (rsum4_n) lane group g
// holds entity 4i + g of batch i, so a lane keeps NB = ceil(NE / 4) probabilities
// per head, not NE + 1.
template <int NE>
constexpr int agent_nb() { return (NE + 3) / 4; }

template <int E, int H, int NE, int FF, bool LEAN>
struct AgentCacheT {
  static constexpr int ET = E / 16, HET = H * ET, NB = agent_nb<NE>();
  typename std::conditional<LEAN, PostCacheLean<E, H, FF>, PostCache<E, H, FF>>::type post;
  f4 u[HET];
  float p0[H];      // probability of token 0 (the hidden state)
  float pr[H][NB];  // entity probabilities, scattered: lane group g holds entity 4i + g
  f4 oh[H];
  float Ps[H];
};
template <int E, int H, int NE, int FF>
using AgentCache = AgentCacheT<E, H, NE, FF, false>;
// lean (PostCacheLean) cache of the two-wave pipelined BPTT: the record's X, Z, Y
// fields are written by the recompute, which is the lighter of the two phases
template <int E, int H, int NE, int FF>
using AgentCacheLean = AgentCacheT<E, H, NE, FF, true>;

// Attention half of block d: u = M x, per head softmax over [h, entities] and
// z_h = p0 h + We ô_h + P_h b_e.  Caches (u, p, ô, P) when C is non-null.
// ne: the entity count (NE, or fewer in a runtime-entity instance: entities
// j >= ne are padding — zero observations, score -inf, probability 0).
template <int E, int H, int NE, int FF, bool LEAN, typename WT>
T2O_DEV void agent_attn_fwd(const Wts<WT>& P, const t2o_layout& L, int d, const f4* h, const f4 (&o)[NE], int ne,
                            const f4* x, f4* z, AgentCacheT<E, H, NE, FF, LEAN>* cache) {
  constexpr int ET = E / 16, HET = H * ET, NB = agent_nb<NE>();
  const float* be = P.v + L.be;
  const int g = lane_g();
  f4 u[HET];
  matvec<HET, ET>(P.w + L.M[d], E, x, u, P.vol);
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    f4 w;
    matvec<1, ET>(P.w + L.WeT, E, &u[hh * ET], &w, P.vol);
    float cpart = 0.f, s0part = 0.f;
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      const f4 bt = vec_t(be, t);
      const f4 ut = u[hh * ET + t];
      cpart += dot4_pk(ut, bt);
      s0part += dot4_pk(ut, h[t]);
    }
    float cs[2] = {cpart, s0part};  // [c, s_0] in every lane
    allsum4_n(cs);
    // entity scores w·o_j reduce-scattered: lane group g gets entity 4i + g, so the
    // softmax's max / exp / sum run on NB values per lane instead of NE + 1
    float sp[4 * NB], s[NB];
#pragma unroll
    for (int j = 0; j < 4 * NB; ++j)
      sp[j] = j < NE ? dot4_pk(w, o[j]) : 0.f;
    rsum4_n(sp, s);
    const float cval = cs[0], s0 = cs[1];
    float m = s0;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      s[i] = 4 * i + g < ne ? s[i] + cval : -INFINITY;
      m = fmaxf(m, s[i]);
    }
    m = allmax4(m);
    const float e0 = exp_fast(s0 - m);
    float lp = 0.f;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      s[i] = exp_fast(s[i] - m);
      lp += s[i];
    }
    const float le = allsum4(lp);  // Σ over the entities
    const float il = rcp_fast(e0 + le);
    const float p0 = e0 * il, Ps = le * il;
#pragma unroll
    for (int i = 0; i < NB; ++i) s[i] *= il;
    float pa[4 * NB];  // every entity's probability in every lane (ô = Σ p_j o_j)
    bcast4_n(s, pa);
    f4 oh = zero4();
#pragma unroll
    for (int j = 0; j < NE; ++j) oh += pa[j] * o[j];
    f4 zz[ET];
    matvec<ET, 1>(P.w + L.We, 16, &oh, zz, P.vol);
#pragma unroll
    for (int t = 0; t < ET; ++t) z[hh * ET + t] = zz[t] + p0 * h[t] + Ps * vec_t(be, t);
    if (cache) {
      cache->oh[hh] = oh;
      cache->Ps[hh] = Ps;
      cache->p0[hh] = p0;
#pragma unroll
      for (int i = 0; i < NB; ++i) cache->pr[hh][i] = s[i];
    }
  }
  if (cache) {
#pragma unroll
    for (int t = 0; t < HET; ++t) cache->u[t] = u[t];
  }
}

// Forward of block d.  h: hidden token (layer-0 key 0), o: observations,
// x: in = block input query, out = block output.
template <int E, int H, int NE, int FF, bool CACHE, typename WT>
T2O_DEV void agent_block_fwd(const Wts<WT>& P, const t2o_layout& L, int d, const f4* h,
                             const f4 (&o)[NE], int ne, f4* x, AgentCache<E, H, NE, FF>* cache) {
  constexpr int HET = H * (E / 16);
  f4 z[HET];
  agent_attn_fwd<E, H, NE, FF, false>(P, L, d, h, o, ne, x, z, CACHE ? cache : nullptr);
  T2O_MARK(2);
  post_fwd<E, H, FF, CACHE>(P, L, d, z, x, CACHE ? &cache->post : nullptr);
}

template <int E, int H, int NE, int FF, typename WT>
T2O_DEV void agent_block_fwd_lean(const Wts<WT>& P, const t2o_layout& L, int d, const f4* h, const f4 (&o)[NE],
                                  int ne, f4* x, AgentCacheLean<E, H, NE, FF>& cache, const MaskedRec<WT>& rec) {
  constexpr int HET = H * (E / 16);
  f4 z[HET];
  agent_attn_fwd<E, H, NE, FF, true>(P, L, d, h, o, ne, x, z, &cache);
  T2O_MARK(2);
  post_fwd_lean<E, H, FF>(P, L, d, z, x, &cache.post, rec);
}

// Register-accumulating variant of the lean pair (the pipelined bf16 BPTT):
// dM = Σ gu ⊗ x and dN = Σ gres ⊗ z stay in MFMA accumulator registers over the
// whole unroll instead of going to the tape (record TapeRecA), and no weight
// gradient is contracted on the dependent chain: the backward phase only
// stages its operands (bf16 tiles of the wave's stage, transposed-read ready:
// gres, gu and per head gz_h, ô_h, u_h, gw_h), and the wave's next phase — a
// recompute, which has slack under the other wave's backward — contracts them
// into dN, dM and dWe (agent_dw_deferred) before staging its own x and z.
// Stage tiles per wave: 0..ET the head's gWo staging (dw_accumulate_regs), z,
// x, gres, gu, then 2(ET+1) per head for dWe.
template <int E, int H>
struct AgentAccTiles {
  static constexpr int ET = E / 16, HET = H * ET;
  static constexpr int ZT = 1 + ET, XT = ZT + HET, GREST = XT + ET, GUT = GREST + ET, WET = GUT + HET;
  static constexpr int WEH = 2 * (ET + 1);  // per head: gz_h (ET), ô_h (1), u_h (ET), gw_h (1)
  static constexpr int N = WET + H * WEH;    // tiles per wave
};

// the weight-grad contractions the previous backward phase of this wave staged
template <int E, int H>
T2O_DEV void agent_dw_deferred(float* __restrict__ stage, f4 (&gM)[H * (E / 16)][E / 16],
                               f4 (&gN)[E / 16][H * (E / 16)], f4 (&gWe)[E / 16][1]) {
  using Tl = AgentAccTiles<E, H>;
  constexpr int ET = Tl::ET, HET = Tl::HET;
  const __bf16* sb = reinterpret_cast<const __bf16*>(stage);
  {  // dN += gres ⊗ z
    bf4 zb[HET];
#pragma unroll
    for (int i = 0; i < HET; ++i) zb[i] = kslice_tile_bf(sb, Tl::ZT + i);
#pragma unroll
    for (int o = 0; o < ET; ++o) {
      const bf4 a = kslice_tile_bf(sb, Tl::GREST + o);
#pragma unroll
      for (int i = 0; i < HET; ++i) gN[o][i] = mfma_b16(a, zb[i], gN[o][i]);
    }
  }
  {  // dM += gu ⊗ x
    bf4 xb[ET];
#pragma unroll
    for (int i = 0; i < ET; ++i) xb[i] = kslice_tile_bf(sb, Tl::XT + i);
#pragma unroll
    for (int o = 0; o < HET; ++o) {
      const bf4 a = kslice_tile_bf(sb, Tl::GUT + o);
#pragma unroll
      for (int i = 0; i < ET; ++i) gM[o][i] = mfma_b16(a, xb[i], gM[o][i]);
    }
  }
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {  // dWe += gz_h ⊗ ô_h + u_h ⊗ gw_h
    const int b = Tl::WET + hh * Tl::WEH;
    const bf4 ob = kslice_tile_bf(sb, b + ET), wb = kslice_tile_bf(sb, b + 2 * ET + 1);
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      gWe[t][0] = mfma_b16(kslice_tile_bf(sb, b + t), ob, gWe[t][0]);
      gWe[t][0] = mfma_b16(kslice_tile_bf(sb, b + ET + 1 + t), wb, gWe[t][0]);
    }
  }
}

template <int E, int H, int NE, int FF, typename WT>
T2O_DEV void agent_block_fwd_acc(const Wts<WT>& P, const t2o_layout& L, int d, const f4* h, const f4 (&o)[NE],
                                 int ne, f4* x, AgentCacheLean<E, H, NE, FF>& cache, const MaskedRec<WT>& rec,
                                 float* __restrict__ stage, f4 (&gM)[H * (E / 16)][E / 16],
                                 f4 (&gN)[E / 16][H * (E / 16)], f4 (&gWe)[E / 16][1]) {
  using Tl = AgentAccTiles<E, H>;
  agent_dw_deferred<E, H>(stage, gM, gN, gWe);
  asm volatile("" ::: "memory");  // the staged operands are read before x / z overwrite theirs
  __bf16* sb = reinterpret_cast<__bf16*>(stage);
#pragma unroll
  for (int t = 0; t < Tl::ET; ++t) stage_tile_bf(sb, Tl::XT + t, x[t]);
  f4 z[Tl::HET];
  agent_attn_fwd<E, H, NE, FF, true>(P, L, d, h, o, ne, x, z, &cache);
#pragma unroll
  for (int t = 0; t < Tl::HET; ++t) stage_tile_bf(sb, Tl::ZT + t, z[t]);
  post_fwd_lean<E, H, FF, WT, TapeRecA<E, H, FF>>(P, L, d, z, x, &cache.post, rec);
}

// Attention half of the backward: from gz (grad wrt z) to gu (grad wrt u = M x);
// gh_in accumulates the grad wrt h through the key/value path (token 0), gbe the
// grad wrt the embedding bias, gWe (MFMA register block, [E][16] as ET x 1 tiles)
// the grad wrt the embedding weight.
// DEFER: stage the dWe operands (AgentAccTiles) for agent_dw_deferred instead.
template <int E, int H, int NE, int FF, bool LEAN, typename WT, bool DEFER = false>
T2O_DEV void agent_attn_bwd(const Wts<WT>& P, const t2o_layout& L, float* __restrict__ stage, const f4* h,
                            const f4 (&o)[NE], const AgentCacheT<E, H, NE, FF, LEAN>& c, const f4* gz, f4* gu,
                            f4* gh_in, f4* gbe, f4 (&gWe)[E / 16][1]) {
  constexpr int ET = E / 16;
  constexpr bool BF = sizeof(WT) == 2;
  using Tl = AgentAccTiles<E, H>;
  __bf16* const sb = reinterpret_cast<__bf16*>(stage);
  const float* be = P.v + L.be;
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    const f4* gzh = &gz[hh * ET];
    const f4* uh = &c.u[hh * ET];
    const float p0 = c.p0[hh];
    // z_h = p0 h + We oh + Ps be
    float gp0p = 0.f, gPp = 0.f;
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      const f4 bt = vec_t(be, t);
      gp0p += dot4_pk(gzh[t], h[t]);
      gPp += dot4_pk(gzh[t], bt);
      gh_in[t] += p0 * gzh[t];
      gbe[t] += c.Ps[hh] * gzh[t];
    }
    f4 goh;
    matvec_tr<1, ET>(P, L.We, 16, L.WeT, E, gzh, &goh);
    if constexpr (DEFER) {
      const int b = Tl::WET + hh * Tl::WEH;
#pragma unroll
      for (int t = 0; t < ET; ++t) {
        stage_tile_bf(sb, b + t, gzh[t]);
        stage_tile_bf(sb, b + ET + 1 + t, uh[t]);
      }
      stage_tile_bf(sb, b + ET, c.oh[hh]);
    } else {
      dw_accumulate_regs<ET, 1, BF>(gWe, gzh, &c.oh[hh], stage);
    }
    // softmax backward over [token 0, entities], the entity terms in the forward's
    // scattered form (lane group g: entity 4i + g)
    constexpr int NB = agent_nb<NE>();
    float cs[2] = {gPp, gp0p};
    allsum4_n(cs);
    const float gP = cs[0], gp0 = cs[1];
    float gpart[4 * NB], gq[NB];
#pragma unroll
    for (int j = 0; j < 4 * NB; ++j)
      gpart[j] = j < NE ? dot4_pk(goh, o[j]) : 0.f;
    rsum4_n(gpart, gq);
    float dl = 0.f;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      gq[i] += gP;
      dl += c.pr[hh][i] * gq[i];
    }
    const float dot = p0 * gp0 + allsum4(dl);
    const float gs0 = p0 * (gp0 - dot);
#pragma unroll
    for (int i = 0; i < NB; ++i) gq[i] = c.pr[hh][i] * (gq[i] - dot);
    float gsa[4 * NB], gcl = 0.f;
#pragma unroll
    for (int i = 0; i < NB; ++i) gcl += gq[i];
    const float gc = allsum4(gcl);  // Σ_j gs_j
    bcast4_n(gq, gsa);
    f4 gw = zero4();
#pragma unroll
    for (int j = 0; j < NE; ++j) gw += gsa[j] * o[j];
    // s_h0 = u_h·h ; s_hj = (WeT u_h)·o_j + u_h·be
    f4 t1[ET];
    matvec<ET, 1>(P.w + L.We, 16, &gw, t1, P.vol);
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      gu[hh * ET + t] = t1[t] + gs0 * h[t] + gc * vec_t(be, t);
      gh_in[t] += gs0 * uh[t];
      gbe[t] += gc * uh[t];
    }
    if constexpr (DEFER) stage_tile_bf(sb, Tl::WET + hh * Tl::WEH + 2 * ET + 1, gw);
    else dw_accumulate_regs<ET, 1, BF>(gWe, uh, &gw, stage);
  }
}

// Backward of block d.  gx: in = grad wrt block output, out = grad wrt block
// input (query path).  M's operand pair goes to the tape record (t2o_common.hpp
// TapeRec).
template <int E, int H, int NE, int FF, typename WT>
T2O_DEV void agent_block_bwd(const Wts<WT>& P, const t2o_layout& L, const t2o_layout& G,
                             float* __restrict__ gs, WT* __restrict__ rec, float* __restrict__ stage, int d,
                             const f4* h, const f4 (&o)[NE], const AgentCache<E, H, NE, FF>& c, f4* gx,
                             f4* gh_in, f4* gbe, f4 (&gWe)[E / 16][1], f4* ln2) {
  constexpr int ET = E / 16, HET = H * ET;
  f4 gz[HET], gres[ET];
  post_bwd<E, H, FF>(P, L, G, gs, rec, d, c.post, gx, gz, gres, ln2);
  T2O_MARK(2);
  f4 gu[HET];
  agent_attn_bwd<E, H, NE, FF, false>(P, L, stage, h, o, c, gz, gu, gh_in, gbe, gWe);
  // u = M x
  if (rec) {
    rec_store<TapeRec<E, H, FF>::SIZE, HET>(rec, TapeRec<E, H, FF>::GU, gu);
    rec_store<TapeRec<E, H, FF>::SIZE, ET>(rec, TapeRec<E, H, FF>::X, c.post.x);
  }
  f4 gxp[ET];
  matvec_tr<ET, HET>(P, L.M[d], E, L.MT[d], H * E, gu, gxp);
#pragma unroll
  for (int t = 0; t < ET; ++t) gx[t] = gxp[t] + gres[t];
}

template <int E, int H, int NE, int FF, typename WT>
T2O_DEV void agent_block_bwd_lean(const Wts<WT>& P, const t2o_layout& L, float* __restrict__ gs,
                                  const MaskedRec<WT>& rec, float* __restrict__ stage, int d, const f4* h,
                                  const f4 (&o)[NE], const AgentCacheLean<E, H, NE, FF>& c, f4* gx, f4* gh_in,
                                  f4* gbe, f4 (&gWe)[E / 16][1], f4* ln2) {
  constexpr int ET = E / 16, HET = H * ET;
  f4 gz[HET], gres[ET];
  post_bwd_lean<E, H, FF>(P, L, gs, rec, d, c.post, gx, gz, gres, ln2);
  T2O_MARK(2);
  f4 gu[HET];
  agent_attn_bwd<E, H, NE, FF, true>(P, L, stage, h, o, c, gz, gu, gh_in, gbe, gWe);
  rec.template store<HET>(TapeRec<E, H, FF>::GU, gu);
  f4 gxp[ET];
  matvec_tr<ET, HET>(P, L.M[d], E, L.MT[d], H * E, gu, gxp);
#pragma unroll
  for (int t = 0; t < ET; ++t) gx[t] = gxp[t] + gres[t];
}

template <int E, int H, int NE, int FF, typename WT>
T2O_DEV void agent_block_bwd_acc(const Wts<WT>& P, const t2o_layout& L, float* __restrict__ gs,
                                 const MaskedRec<WT>& rec, float* __restrict__ stage, int d, const f4* h,
                                 const f4 (&o)[NE], const AgentCacheLean<E, H, NE, FF>& c, f4* gx, f4* gh_in,
                                 f4* gbe, f4 (&gWe)[E / 16][1], f4* ln2, f4 (&gM)[H * (E / 16)][E / 16],
                                 f4 (&gN)[E / 16][H * (E / 16)]) {
  using Tl = AgentAccTiles<E, H>;
  constexpr int ET = E / 16, HET = H * ET;
  __bf16* const sb = reinterpret_cast<__bf16*>(stage);
  f4 gz[HET], gres[ET];
  post_bwd_lean<E, H, FF, WT, TapeRecA<E, H, FF>>(P, L, gs, rec, d, c.post, gx, gz, gres, ln2);
#pragma unroll
  for (int t = 0; t < ET; ++t) stage_tile_bf(sb, Tl::GREST + t, gres[t]);  // dN += gres ⊗ z, deferred
  T2O_MARK(2);
  f4 gu[HET];
  agent_attn_bwd<E, H, NE, FF, true, WT, true>(P, L, stage, h, o, c, gz, gu, gh_in, gbe, gWe);
#pragma unroll
  for (int t = 0; t < HET; ++t) stage_tile_bf(sb, Tl::GUT + t, gu[t]);  // dM += gu ⊗ x, deferred
  f4 gxp[ET];
  matvec_tr<ET, HET>(P, L.M[d], E, L.MT[d], H * E, gu, gxp);
#pragma unroll
  for (int t = 0; t < ET; ++t) gx[t] = gxp[t] + gres[t];
}

}  // namespace t2o
