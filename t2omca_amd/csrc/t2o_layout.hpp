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
__host__ __device__ constexpr void grad_layout(const t2o_layout& L, t2o_layout& G) {
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

// Offsets of the folded MFMA pack of a tuned network — forward matrices, then
// forward vectors (one contiguous LDS copy; in bf16 mode the vectors stay fp32),
// then the backward's transposed copies; every size a multiple of 16 elements, so
// every section stays 64-B aligned.  They depend on (E, H, D, FF, prec) only.
// ONE definition: t2o_layout_init_ex fills a caller's layout with it, and the
// tuned kernels instantiate it as a compile-time constant (kernel_layout), so
// every offset is an immediate there instead of a 64-bit kernel argument held in
// SGPRs (the BPTT kernels spilled 70-170 SGPRs to VGPR lanes holding them).
__host__ __device__ constexpr void tuned_pack_offsets(t2o_layout& L, int E, int H, int D, int FF, int prec) {
  int64_t o = 0;
  const int64_t HE = (int64_t)H * E;
  L.WeT = o; o += 16 * (int64_t)E;
  L.We = o; o += (int64_t)E * 16;
  L.Wo = o; o += 16 * (int64_t)E;
  for (int d = 0; d < D; ++d) {
    L.M[d] = o; o += HE * E;
    L.N[d] = o; o += E * HE;
    L.W1[d] = o; o += (int64_t)FF * E;
    L.W2[d] = o; o += (int64_t)E * FF;
  }
  L.vec_lo = o;
  L.be = o; o += E;
  L.bo = o; o += 16;
  for (int d = 0; d < D; ++d) {
    L.bu[d] = o; o += E;
    L.g1[d] = o; o += E;
    L.n1[d] = o; o += E;
    L.c1[d] = o; o += FF;
    L.c2[d] = o; o += E;
    L.g2[d] = o; o += E;
    L.n2[d] = o; o += E;
  }
  L.fwd_total = o;
  L.WoT = o; o += (int64_t)E * 16;
  for (int d = 0; d < D; ++d) {
    L.MT[d] = o; o += E * HE;
    L.NT[d] = o; o += HE * E;
    L.W1T[d] = o; o += (int64_t)E * FF;
    L.W2T[d] = o; o += (int64_t)FF * E;
  }
  L.total = o;
  L.pack_floats = prec ? o + ((o + 1) / 2 + 3) / 4 * 4 : o;
  t2o_layout G{};
  grad_layout(L, G);
  L.grad_total = G.grad_total;
}

template <int E, int H, int D, int FF, int PREC>
__host__ __device__ constexpr t2o_layout tuned_layout_const() {
  t2o_layout L{};
  L.E = E; L.H = H; L.D = D; L.FF = FF; L.prec = PREC;
  for (int d = 0; d < T2O_MAX_DEPTH; ++d)
    L.M[d] = L.MT[d] = L.N[d] = L.NT[d] = L.bu[d] = L.g1[d] = L.n1[d] = L.W1[d] = L.W1T[d] = L.c1[d] =
        L.W2[d] = L.W2T[d] = L.c2[d] = L.g2[d] = L.n2[d] = -1;
  tuned_pack_offsets(L, E, H, D, FF, PREC);
  return L;
}

// A tuned kernel's layout: the compile-time pack offsets of its instance with
// the caller's run-time scalars (kind, feature / action / entity counts, mixer
// head).  The launchers check the caller's offsets equal the constant ones
// (kernel_layout_matches), so the two can never disagree silently.
template <int E, int H, int D, int FF, typename WT>
__host__ __device__ inline t2o_layout kernel_layout(const t2o_layout& rt) {
  constexpr t2o_layout C = tuned_layout_const<E, H, D, FF, sizeof(WT) == 2>();
  t2o_layout L = C;
  L.kind = rt.kind; L.F = rt.F; L.NA = rt.NA; L.n_ent = rt.n_ent; L.n_agents = rt.n_agents;
  L.pos_func = rt.pos_func; L.pos_beta = rt.pos_beta;
  return L;
}
template <int E, int H, int D, int FF, int PREC>
__host__ __device__ constexpr t2o_layout tuned_grad_layout_const() {
  const t2o_layout C = tuned_layout_const<E, H, D, FF, PREC>();
  t2o_layout G{};
  grad_layout(C, G);
  return G;
}
template <int E, int H, int D, int FF, typename WT>
__host__ __device__ inline t2o_layout kernel_grad_layout() {
  constexpr t2o_layout G = tuned_grad_layout_const<E, H, D, FF, sizeof(WT) == 2>();
  return G;
}
template <int E, int H, int D, int FF, typename WT>
inline bool kernel_layout_matches(const t2o_layout& rt) {
  constexpr t2o_layout C = tuned_layout_const<E, H, D, FF, sizeof(WT) == 2>();
  bool ok = rt.WeT == C.WeT && rt.We == C.We && rt.be == C.be && rt.Wo == C.Wo && rt.bo == C.bo &&
            rt.WoT == C.WoT && rt.fwd_total == C.fwd_total && rt.total == C.total &&
            rt.grad_total == C.grad_total && rt.vec_lo == C.vec_lo && rt.pack_floats == C.pack_floats && !rt.generic;
  for (int d = 0; d < D; ++d)
    ok = ok && rt.M[d] == C.M[d] && rt.MT[d] == C.MT[d] && rt.N[d] == C.N[d] && rt.NT[d] == C.NT[d] &&
         rt.bu[d] == C.bu[d] && rt.g1[d] == C.g1[d] && rt.n1[d] == C.n1[d] && rt.W1[d] == C.W1[d] &&
         rt.W1T[d] == C.W1T[d] && rt.c1[d] == C.c1[d] && rt.W2[d] == C.W2[d] && rt.W2T[d] == C.W2T[d] &&
         rt.c2[d] == C.c2[d] && rt.g2[d] == C.g2[d] && rt.n2[d] == C.n2[d];
  return ok;
}

}  // namespace t2o
