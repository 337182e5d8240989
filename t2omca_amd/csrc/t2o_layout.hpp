// t2o_layout.hpp — host/device description of parameter, pack and gradient layouts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/t2omca.h"

namespace t2o {

// Offsets (floats) of the reference parameters in state_dict order
// (transf_agent.py:9-48, n_transf_mixer.py:13-53, transformer.py:34-38,103-118).
struct ParamOffsets {
  int64_t We, be;
  int64_t Wk[T2O_MAX_DEPTH], Wq[T2O_MAX_DEPTH], Wv[T2O_MAX_DEPTH], U[T2O_MAX_DEPTH], bu[T2O_MAX_DEPTH];
  int64_t g1[T2O_MAX_DEPTH], n1[T2O_MAX_DEPTH], g2[T2O_MAX_DEPTH], n2[T2O_MAX_DEPTH];
  int64_t W1[T2O_MAX_DEPTH], c1[T2O_MAX_DEPTH], W2[T2O_MAX_DEPTH], c2[T2O_MAX_DEPTH];
  int64_t Wo, bo;  // q_basic (agent) or hyper_b2 (mixer)
  int64_t total;
};

__host__ __device__ inline ParamOffsets param_offsets(int kind, int E, int H, int D, int F, int NA, int FF) {
  ParamOffsets p{};
  int64_t o = 0;
  const int64_t HE = (int64_t)H * E;
  p.We = o; o += (int64_t)E * F;
  p.be = o; o += E;
  for (int d = 0; d < D; ++d) {
    p.Wk[d] = o; o += HE * E;
    p.Wq[d] = o; o += HE * E;
    p.Wv[d] = o; o += HE * E;
    p.U[d] = o; o += E * HE;
    p.bu[d] = o; o += E;
    p.g1[d] = o; o += E;
    p.n1[d] = o; o += E;
    p.g2[d] = o; o += E;
    p.n2[d] = o; o += E;
    p.W1[d] = o; o += (int64_t)FF * E;
    p.c1[d] = o; o += FF;
    p.W2[d] = o; o += (int64_t)E * FF;
    p.c2[d] = o; o += E;
  }
  const int no = kind == 0 ? NA : 1;
  p.Wo = o; o += (int64_t)no * E;
  p.bo = o; o += no;
  p.total = o;
  return p;
}

// ---- runtime-shaped ("generic") networks (t2o_generic.hip) -------------------
// Pack: the reference-order parameters [0, P.total), then transposed copies, so
// that every lane-per-feature matrix-vector product of the generic kernels reads
// its weights coalesced (lane = output feature, consecutive lanes = consecutive
// addresses): forward q = Wq x, v = Wv z, a = U v, f1 = W1 y, r2 = W2 fr, the
// entity embedding and the agent head read the transposes; backward products
// read the originals, except gq = Wk gu (transpose of u = Wkᵀ q) which reads WkT.
struct GenOffsets {
  ParamOffsets P;
  int64_t WqT[T2O_MAX_DEPTH], WkT[T2O_MAX_DEPTH], WvT[T2O_MAX_DEPTH];  // [E][HE]
  int64_t UT[T2O_MAX_DEPTH];                                          // [HE][E]
  int64_t W1T[T2O_MAX_DEPTH];                                         // [E][FF]
  int64_t W2T[T2O_MAX_DEPTH];                                         // [FF][E]
  int64_t WeT, WoT;                                                   // [F][E], [E][no]
  int64_t total;
};

__host__ __device__ inline GenOffsets gen_offsets(int kind, int E, int H, int D, int F, int NA, int FF) {
  GenOffsets g{};
  g.P = param_offsets(kind, E, H, D, F, NA, FF);
  int64_t o = g.P.total;
  const int64_t HE = (int64_t)H * E;
  for (int d = 0; d < D; ++d) {
    g.WqT[d] = o; o += E * HE;
    g.WkT[d] = o; o += E * HE;
    g.WvT[d] = o; o += E * HE;
    g.UT[d] = o; o += HE * E;
    g.W1T[d] = o; o += (int64_t)E * FF;
    g.W2T[d] = o; o += (int64_t)FF * E;
  }
  g.WeT = o; o += (int64_t)F * E;
  g.WoT = o; o += (int64_t)E * (kind == 0 ? NA : 1);
  g.total = o;
  return g;
}

// Generic weight-gradient record of one (row, step, block): the operand vectors
// of dWq = Σ gq⊗x, dWk_h = Σ q_h⊗gu_h, dWv_h = Σ gv_h⊗z_h, dU = Σ ga⊗v,
// dW1 = Σ gf1⊗y, dW2 = Σ gr2⊗relu(f1) (fp32; contracted by t2o_generic.hip).
struct GenRec {
  int X, Q, GQ, GU, Z, GV, V, GA, Y, GF1, GR2, FR, SIZE;
};
__host__ __device__ inline GenRec gen_rec(int E, int H, int FF) {
  GenRec r{};
  const int HE = H * E;
  int o = 0;
  r.X = o; o += E;
  r.Q = o; o += HE;
  r.GQ = o; o += HE;
  r.GU = o; o += HE;
  r.Z = o; o += HE;
  r.GV = o; o += HE;
  r.V = o; o += HE;
  r.GA = o; o += E;
  r.Y = o; o += E;
  r.GF1 = o; o += FF;
  r.GR2 = o; o += E;
  r.FR = o; o += FF;
  r.SIZE = (o + 3) / 4 * 4;
  return r;
}

// Records per weight-gradient tape tile (TapeRec, t2o_common.hpp): 16 — one
// wave's rows (agent), or 16 consecutive records of a tuned mixer's compact
// per-block stream of query-row records (no padding records in HBM).
inline int tape_tile_records(const t2o_layout&) { return 16; }

// Compact gradient layout (what the backward kernels accumulate in LDS and
// write per workgroup): the pack layout without transposed copies.
inline void grad_layout(const t2o_layout& L, t2o_layout& G) {
  G = L;
  int64_t o = 0;
  const int64_t E = L.E, HE = (int64_t)L.H * L.E, FF = L.FF;
  G.We = o; o += E * 16;
  G.be = o; o += E;
  G.Wo = o; o += 16 * E;
  G.bo = o; o += 16;
  G.WeT = G.WoT = -1;
  for (int d = 0; d < T2O_MAX_DEPTH; ++d) {
    G.MT[d] = G.NT[d] = G.W1T[d] = G.W2T[d] = -1;
    if (d >= L.D) { G.M[d] = G.N[d] = G.bu[d] = G.g1[d] = G.n1[d] = G.W1[d] = G.c1[d] = G.W2[d] = G.c2[d] = G.g2[d] = G.n2[d] = -1; continue; }
    G.M[d] = o; o += HE * E;
    G.N[d] = o; o += E * HE;
    G.bu[d] = o; o += E;
    G.g1[d] = o; o += E;
    G.n1[d] = o; o += E;
    G.W1[d] = o; o += FF * E;
    G.c1[d] = o; o += FF;
    G.W2[d] = o; o += E * FF;
    G.c2[d] = o; o += E;
    G.g2[d] = o; o += E;
    G.n2[d] = o; o += E;
  }
  G.total = G.grad_total = G.fwd_total = o;
}

}  // namespace t2o
