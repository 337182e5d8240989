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
//   a = Σ_h N_h z_h + b_U;  y = LN1(a + x);  x' = LN2(W2 relu(W1 y + c1) + c2 + y)
// Observation features live in the T-layout over a 16-padded F axis: lane
// group g holds o_j[4g .. 4g+3], so every per-entity dot product is 4 FMAs
// plus a 4-lane all-reduce.
#pragma once
#include "t2o_common.hpp"

namespace t2o {

template <int E, int H, int NE, int FF>
struct AgentCache {
  static constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
  f4 x[ET];
  f4 u[HET];
  float p[H][NE + 1];
  f4 oh[H];
  float Ps[H];
  f4 z[HET];
  f4 xh1[ET];
  float rs1;
  f4 y[ET];
  f4 f1[FT];
  f4 xh2[ET];
  float rs2;
};

// Forward of block d.  h: hidden token (layer-0 key 0), o: observations,
// x: in = block input query, out = block output.
template <int E, int H, int NE, int FF, bool CACHE>
T2O_DEV void agent_block_fwd(const float* __restrict__ P, const t2o_layout& L, int d, const f4* h,
                             const f4 (&o)[NE], f4* x, AgentCache<E, H, NE, FF>* cache) {
  constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
  const float* be = P + L.be;
  f4 u[HET];
  matvec<HET, ET>(P + L.M[d], E, x, u);
  float p[H][NE + 1];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    f4 w;
    matvec<1, ET>(P + L.WeT, E, &u[hh * ET], &w);
    float cpart = 0.f, s0part = 0.f;
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      const f4 bt = vec_t(be, t);
      const f4 ut = u[hh * ET + t];
      cpart += (ut[0] * bt[0] + ut[1] * bt[1]) + (ut[2] * bt[2] + ut[3] * bt[3]);
      s0part += (ut[0] * h[t][0] + ut[1] * h[t][1]) + (ut[2] * h[t][2] + ut[3] * h[t][3]);
    }
    const float cval = allsum4(cpart);
    p[hh][0] = allsum4(s0part);
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const float sp = (w[0] * o[j][0] + w[1] * o[j][1]) + (w[2] * o[j][2] + w[3] * o[j][3]);
      p[hh][j + 1] = allsum4(sp) + cval;
    }
    float m = p[hh][0];
#pragma unroll
    for (int j = 1; j <= NE; ++j) m = fmaxf(m, p[hh][j]);
    float l = 0.f;
#pragma unroll
    for (int j = 0; j <= NE; ++j) {
      p[hh][j] = expf(p[hh][j] - m);
      l += p[hh][j];
    }
    const float il = 1.0f / l;
#pragma unroll
    for (int j = 0; j <= NE; ++j) p[hh][j] *= il;
  }
  f4 z[HET];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    f4 oh = zero4();
    float Ps = 0.f;
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      oh += p[hh][j + 1] * o[j];
      Ps += p[hh][j + 1];
    }
    f4 zz[ET];
    matvec<ET, 1>(P + L.We, 16, &oh, zz);
#pragma unroll
    for (int t = 0; t < ET; ++t) z[hh * ET + t] = zz[t] + p[hh][0] * h[t] + Ps * vec_t(be, t);
    if constexpr (CACHE) {
      cache->oh[hh] = oh;
      cache->Ps[hh] = Ps;
#pragma unroll
      for (int j = 0; j <= NE; ++j) cache->p[hh][j] = p[hh][j];
    }
  }
  f4 r1[ET];
  matvec<ET, HET>(P + L.N[d], H * E, z, r1);
#pragma unroll
  for (int t = 0; t < ET; ++t) r1[t] += vec_t(P + L.bu[d], t) + x[t];
  f4 y[ET], xh1[ET];
  float rs1;
  layernorm_fwd<ET>(r1, P + L.g1[d], P + L.n1[d], y, xh1, rs1);
  f4 f1[FT];
  matvec<FT, ET>(P + L.W1[d], E, y, f1);
  f4 f1r[FT];
#pragma unroll
  for (int t = 0; t < FT; ++t) {
    f1[t] += vec_t(P + L.c1[d], t);
#pragma unroll
    for (int r = 0; r < 4; ++r) f1r[t][r] = fmaxf(f1[t][r], 0.f);
  }
  f4 r2[ET];
  matvec<ET, FT>(P + L.W2[d], FF, f1r, r2);
#pragma unroll
  for (int t = 0; t < ET; ++t) r2[t] += vec_t(P + L.c2[d], t) + y[t];
  if constexpr (CACHE) {
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      cache->x[t] = x[t];
      cache->xh1[t] = xh1[t];
      cache->y[t] = y[t];
    }
#pragma unroll
    for (int t = 0; t < HET; ++t) {
      cache->u[t] = u[t];
      cache->z[t] = z[t];
    }
#pragma unroll
    for (int t = 0; t < FT; ++t) cache->f1[t] = f1[t];
    cache->rs1 = rs1;
  }
  f4 xh2[ET];
  float rs2;
  layernorm_fwd<ET>(r2, P + L.g2[d], P + L.n2[d], x, xh2, rs2);
  if constexpr (CACHE) {
#pragma unroll
    for (int t = 0; t < ET; ++t) cache->xh2[t] = xh2[t];
    cache->rs2 = rs2;
  }
}


// Backward of block d.  gx: in = grad wrt block output, out = grad wrt block
// input (query path).  gh_in accumulates the grad wrt h through the key/value
// path (token 0).  Weight grads are accumulated into the LDS gradient block G
// (compact layout, t2o_layout.hpp) over the wave's 16 rows.
template <int E, int H, int NE, int FF>
T2O_DEV void agent_block_bwd(const float* __restrict__ P, const t2o_layout& L, const t2o_layout& G,
                             float* __restrict__ lg, float* __restrict__ stage, int d, const f4* h,
                             const f4 (&o)[NE], const AgentCache<E, H, NE, FF>& c, f4* gx, f4* gh_in,
                             f4* gbe) {
  constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
  const float* be = P + L.be;
  // ---- LN2: x' = xh2*g2 + n2
  {
    f4 t0[ET];
#pragma unroll
    for (int t = 0; t < ET; ++t) t0[t] = gx[t] * c.xh2[t];
    vec_accumulate<ET>(lg + G.g2[d], t0);
    vec_accumulate<ET>(lg + G.n2[d], gx);
  }
  f4 gr2[ET];
  layernorm_bwd<ET>(gx, c.xh2, c.rs2, P + L.g2[d], gr2);
  // ---- FFN: r2 = W2 relu(f1) + c2 + y
  {
    f4 f1r[FT];
#pragma unroll
    for (int t = 0; t < FT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) f1r[t][r] = fmaxf(c.f1[t][r], 0.f);
    dw_accumulate<ET, FT>(lg + G.W2[d], FF, gr2, f1r, stage);
  }
  vec_accumulate<ET>(lg + G.c2[d], gr2);
  f4 gf1[FT];
  matvec<FT, ET>(P + L.W2T[d], E, gr2, gf1);
#pragma unroll
  for (int t = 0; t < FT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) gf1[t][r] = c.f1[t][r] > 0.f ? gf1[t][r] : 0.f;
  dw_accumulate<FT, ET>(lg + G.W1[d], E, gf1, c.y, stage);
  vec_accumulate<FT>(lg + G.c1[d], gf1);
  f4 gy[ET];
  matvec<ET, FT>(P + L.W1T[d], FF, gf1, gy);
#pragma unroll
  for (int t = 0; t < ET; ++t) gy[t] += gr2[t];
  // ---- LN1: y = xh1*g1 + n1
  {
    f4 t0[ET];
#pragma unroll
    for (int t = 0; t < ET; ++t) t0[t] = gy[t] * c.xh1[t];
    vec_accumulate<ET>(lg + G.g1[d], t0);
    vec_accumulate<ET>(lg + G.n1[d], gy);
  }
  f4 gr1[ET];
  layernorm_bwd<ET>(gy, c.xh1, c.rs1, P + L.g1[d], gr1);
  // ---- r1 = N z + b_U + x
  dw_accumulate<ET, HET>(lg + G.N[d], H * E, gr1, c.z, stage);
  vec_accumulate<ET>(lg + G.bu[d], gr1);
  f4 gz[HET];
  matvec<HET, ET>(P + L.NT[d], E, gr1, gz);
  f4 gu[HET];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    const f4* gzh = &gz[hh * ET];
    const f4* uh = &c.u[hh * ET];
    const float p0 = c.p[hh][0];
    // z_h = p0 h + We oh + Ps be
    float gp0p = 0.f, gPp = 0.f;
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      const f4 bt = vec_t(be, t);
      gp0p += (gzh[t][0] * h[t][0] + gzh[t][1] * h[t][1]) + (gzh[t][2] * h[t][2] + gzh[t][3] * h[t][3]);
      gPp += (gzh[t][0] * bt[0] + gzh[t][1] * bt[1]) + (gzh[t][2] * bt[2] + gzh[t][3] * bt[3]);
      gh_in[t] += p0 * gzh[t];
      gbe[t] += c.Ps[hh] * gzh[t];
    }
    const float gp0 = allsum4(gp0p);
    const float gP = allsum4(gPp);
    f4 goh;
    matvec<1, ET>(P + L.WeT, E, gzh, &goh);
    dw_accumulate<ET, 1>(lg + G.We, 16, gzh, &c.oh[hh], stage);
    // softmax backward over [token 0, entities]
    float gp[NE + 1];
    gp[0] = gp0;
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const float sp = (goh[0] * o[j][0] + goh[1] * o[j][1]) + (goh[2] * o[j][2] + goh[3] * o[j][3]);
      gp[j + 1] = allsum4(sp) + gP;
    }
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j <= NE; ++j) dot += c.p[hh][j] * gp[j];
    const float gs0 = p0 * (gp[0] - dot);
    f4 gw = zero4();
    float gc = 0.f;
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const float gsj = c.p[hh][j + 1] * (gp[j + 1] - dot);
      gw += gsj * o[j];
      gc += gsj;
    }
    // s_h0 = u_h·h ; s_hj = (WeT u_h)·o_j + u_h·be
    f4 t1[ET];
    matvec<ET, 1>(P + L.We, 16, &gw, t1);
#pragma unroll
    for (int t = 0; t < ET; ++t) {
      gu[hh * ET + t] = t1[t] + gs0 * h[t] + gc * vec_t(be, t);
      gh_in[t] += gs0 * uh[t];
      gbe[t] += gc * uh[t];
    }
    dw_accumulate<ET, 1>(lg + G.We, 16, uh, &gw, stage);
  }
  // ---- u = M x
  dw_accumulate<HET, ET>(lg + G.M[d], E, gu, c.x, stage);
  f4 gxp[ET];
  matvec<ET, HET>(P + L.MT[d], H * E, gu, gxp);
#pragma unroll
  for (int t = 0; t < ET; ++t) gx[t] = gxp[t] + gr1[t];
}

}  // namespace t2o
