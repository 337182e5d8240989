// t2o_agent_block_ch.hpp — the agent block for many entities (n_ent > 16):
// the same algebra as t2o_agent_block.hpp, but the observations are streamed
// from memory in chunks of AG_CHUNK entities with an online softmax (running
// max / sum per head, accumulators rescaled per chunk) instead of being held
// in registers, and the backward recomputes the probabilities chunk by chunk
// from the cached per-head (w, c, max, 1/sum) instead of caching them.
//
// Reference: transformer.py:40-140 via transf_agent.py:54-76 (n_entities =
// n_agents, environment_multi_mec.py:429), BASELINE configs[3] at 64 AGVs.
//
// Softmax backward without a pass for the normaliser term:
//   dot_h = Σ_j p_j gp_j = p_0 gp_0 + goh_h·ô_h + gP_h P_h
// (gp_j = goh_h·o_j + gP_h for entities), so one chunk pass per block
// produces gw_h = Σ_j gs_j o_j and gc_h = Σ_j gs_j with gs_j = p_j (gp_j - dot_h).
#pragma once
#include "t2o_block.hpp"

namespace t2o {

constexpr int AG_CHUNK = 8;
// entity counts above this take the streamed path
#ifndef T2O_AG_CHUNK_MIN
#define T2O_AG_CHUNK_MIN 16
#endif
constexpr int AG_CHUNK_MIN = T2O_AG_CHUNK_MIN;

// One row's observation vector in memory: entity j, feature f at ob[j*F + f];
// a lane loads the T-layout slice (features 4g .. 4g+3, zero-padded past F).
// ne entities; `tail` when ne is not a multiple of the chunk (a runtime-entity
// instance): the last chunk's entities j >= ne load zeros and score -inf.
struct ObsRow {
  const float* ob;
  int F;
  int ne;
  bool tail;
  template <int CH>
  T2O_DEV void load(int j0, f4 (&o)[CH]) const {
    const int g = lane_g();
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 4 * g + r;
        o[j][r] = (f < F && (!tail || j0 + j < ne)) ? ob[(j0 + j) * F + f] : 0.f;
      }
  }
  T2O_DEV bool pad(int j) const { return tail && j >= ne; }
};

template <int E, int H, int NE, int FF>
struct AgentCacheCh {
  static constexpr int ET = E / 16, HET = H * ET;
  PostCache<E, H, FF> post;
  f4 u[HET];
  f4 w[H];          // We_ᵀ u_h (observation space)
  float cval[H];    // u_h · b_e
  float m[H];       // running max of the head's scores (final)
  float il[H];      // 1 / Σ exp(s - m)
  float p0[H];      // probability of token 0 (the hidden state)
  f4 oh[H];         // Σ_j p_j o_j
  float Ps[H];      // Σ_j p_j
};

template <int E, int H, int NE, int FF, bool CACHE, typename WT>
T2O_DEV void agent_block_fwd_ch(const Wts<WT>& P, const t2o_layout& L, int d, const f4* h, const ObsRow& orow,
                                f4* x, AgentCacheCh<E, H, NE, FF>* cache) {
  constexpr int ET = E / 16, HET = H * ET, CH = AG_CHUNK;
  const float* be = P.v + L.be;
  f4 u[HET];
  matvec<HET, ET>(P.w + L.M[d], E, x, u, P.vol);
  f4 w[H], oh[H];
  float cval[H], s0[H], m[H], l[H], e0[H], Ps[H];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    matvec<1, ET>(P.w + L.WeT, E, &u[hh * ET], &w[hh], P.vol);
    float cpart = 0.f, s0part = 0.f;
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      const f4 bt = vec_t(be, t);
      const f4 ut = u[hh * ET + t];
      cpart += (ut[0] * bt[0] + ut[1] * bt[1]) + (ut[2] * bt[2] + ut[3] * bt[3]);
      s0part += (ut[0] * h[t][0] + ut[1] * h[t][1]) + (ut[2] * h[t][2] + ut[3] * h[t][3]);
    }
    cval[hh] = allsum4(cpart);
    s0[hh] = allsum4(s0part);
    m[hh] = s0[hh];
    l[hh] = 1.f;
    e0[hh] = 1.f;
    Ps[hh] = 0.f;
    oh[hh] = zero4();
  }
  f4 o[CH];
  orow.load<CH>(0, o);
  const int ne = orow.ne;
  for (int j0 = 0; j0 < ne; j0 += CH) {
    f4 on[CH];
    if (j0 + CH < ne) orow.load<CH>(j0 + CH, on);  // next chunk in flight while this one computes
#pragma unroll
    for (int hh = 0; hh < H; ++hh) {
      float s[CH];
      float mc = m[hh];
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const f4 wv = w[hh];
        s[j] = allsum4((wv[0] * o[j][0] + wv[1] * o[j][1]) + (wv[2] * o[j][2] + wv[3] * o[j][3])) + cval[hh];
        if (orow.pad(j0 + j)) s[j] = -INFINITY;
        mc = fmaxf(mc, s[j]);
      }
      const float sc = exp_fast(m[hh] - mc);
      l[hh] *= sc;
      e0[hh] *= sc;
      Ps[hh] *= sc;
      oh[hh] *= sc;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const float e = exp_fast(s[j] - mc);
        l[hh] += e;
        Ps[hh] += e;
        oh[hh] += e * o[j];
      }
      m[hh] = mc;
    }
    if (j0 + CH < ne) {
#pragma unroll
      for (int j = 0; j < CH; ++j) o[j] = on[j];
    }
  }
  f4 z[HET];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    const float il = rcp_fast(l[hh]);
    const float p0 = e0[hh] * il;
    oh[hh] *= il;
    Ps[hh] *= il;
    f4 zz[ET];
    matvec<ET, 1>(P.w + L.We, 16, &oh[hh], zz, P.vol);
#pragma unroll
    for (int t = 0; t < ET; ++t) z[hh * ET + t] = zz[t] + p0 * h[t] + Ps[hh] * vec_t(be, t);
    if constexpr (CACHE) {
      cache->w[hh] = w[hh];
      cache->cval[hh] = cval[hh];
      cache->m[hh] = m[hh];
      cache->il[hh] = il;
      cache->p0[hh] = p0;
      cache->oh[hh] = oh[hh];
      cache->Ps[hh] = Ps[hh];
    }
  }
  if constexpr (CACHE) {
#pragma unroll
    for (int t = 0; t < HET; ++t) cache->u[t] = u[t];
  }
  post_fwd<E, H, FF, CACHE>(P, L, d, z, x, CACHE ? &cache->post : nullptr);
}

// Backward of block d (see agent_block_bwd for the argument roles).
template <int E, int H, int NE, int FF, typename WT>
T2O_DEV void agent_block_bwd_ch(const Wts<WT>& P, const t2o_layout& L, const t2o_layout& G,
                                float* __restrict__ gs, WT* __restrict__ rec, float* __restrict__ stage, int d,
                                const f4* h, const ObsRow& orow, const AgentCacheCh<E, H, NE, FF>& c, f4* gx,
                                f4* gh_in, f4* gbe, f4 (&gWe)[E / 16][1], f4* ln2) {
  constexpr int ET = E / 16, HET = H * ET, CH = AG_CHUNK;
  constexpr bool BF = sizeof(WT) == 2;
  const float* be = P.v + L.be;
  f4 gz[HET], gres[ET];
  post_bwd<E, H, FF>(P, L, G, gs, rec, d, c.post, gx, gz, gres, ln2);
  f4 goh[H], gw[H];
  float gP[H], dot[H], gs0[H], gc[H];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    const f4* gzh = &gz[hh * ET];
    // z_h = p0 h + We oh + Ps be
    float gp0p = 0.f, gPp = 0.f;
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      const f4 bt = vec_t(be, t);
      gp0p += (gzh[t][0] * h[t][0] + gzh[t][1] * h[t][1]) + (gzh[t][2] * h[t][2] + gzh[t][3] * h[t][3]);
      gPp += (gzh[t][0] * bt[0] + gzh[t][1] * bt[1]) + (gzh[t][2] * bt[2] + gzh[t][3] * bt[3]);
      gh_in[t] += c.p0[hh] * gzh[t];
      gbe[t] += c.Ps[hh] * gzh[t];
    }
    const float gp0 = allsum4(gp0p);
    gP[hh] = allsum4(gPp);
    matvec_tr<1, ET>(P, L.We, 16, L.WeT, E, gzh, &goh[hh]);
    dw_accumulate_regs<ET, 1, BF>(gWe, gzh, &c.oh[hh], stage);
    const f4 go = goh[hh], ohv = c.oh[hh];
    const float goo = allsum4((go[0] * ohv[0] + go[1] * ohv[1]) + (go[2] * ohv[2] + go[3] * ohv[3]));
    dot[hh] = c.p0[hh] * gp0 + goo + gP[hh] * c.Ps[hh];
    gs0[hh] = c.p0[hh] * (gp0 - dot[hh]);
    gw[hh] = zero4();
    gc[hh] = 0.f;
  }
  // entities, chunk by chunk: p recomputed from the cached (w, c, max, 1/sum)
  f4 o[CH];
  orow.load<CH>(0, o);
  const int ne = orow.ne;
  for (int j0 = 0; j0 < ne; j0 += CH) {
    f4 on[CH];
    if (j0 + CH < ne) orow.load<CH>(j0 + CH, on);
#pragma unroll
    for (int hh = 0; hh < H; ++hh) {
      const f4 wv = c.w[hh], go = goh[hh];
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        float s = allsum4((wv[0] * o[j][0] + wv[1] * o[j][1]) + (wv[2] * o[j][2] + wv[3] * o[j][3])) +
                  c.cval[hh];
        if (orow.pad(j0 + j)) s = -INFINITY;
        const float p = exp_fast(s - c.m[hh]) * c.il[hh];
        const float gp =
            allsum4((go[0] * o[j][0] + go[1] * o[j][1]) + (go[2] * o[j][2] + go[3] * o[j][3])) + gP[hh];
        const float gsj = p * (gp - dot[hh]);
        gw[hh] += gsj * o[j];
        gc[hh] += gsj;
      }
    }
    if (j0 + CH < ne) {
#pragma unroll
      for (int j = 0; j < CH; ++j) o[j] = on[j];
    }
  }
  f4 gu[HET];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    const f4* uh = &c.u[hh * ET];
    // s_h0 = u_h·h ; s_hj = (WeT u_h)·o_j + u_h·be
    f4 t1[ET];
    matvec<ET, 1>(P.w + L.We, 16, &gw[hh], t1, P.vol);
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      gu[hh * ET + t] = t1[t] + gs0[hh] * h[t] + gc[hh] * vec_t(be, t);
      gh_in[t] += gs0[hh] * uh[t];
      gbe[t] += gc[hh] * uh[t];
    }
    dw_accumulate_regs<ET, 1, BF>(gWe, uh, &gw[hh], stage);
  }
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

}  // namespace t2o
