// t2o_generic.hip — runtime-shaped TransformerAgent / TransformerMixer unrolls
// (forward + BPTT) and their weight-gradient contraction, for every network
// shape the tuned MFMA kernels are not instantiated for (t2o_layout.generic = 1:
// any emb <= 64, heads <= 8, depth <= 4, ff_hidden_mult, entity / agent counts,
// the mixer's separate state-token count and every qmix_pos_func).
//
// Reference: transformer.py:40-178 (wide heads, keys from the layer-0 input,
// post-LN blocks), transf_agent.py:54-76 (hidden token first, Q from token 0),
// n_transf_mixer.py:55-103 (state tokens, agent hidden tokens, 3 recurrent hyper
// tokens; w1 / b1 / w2 / b2 from the last A+3 output tokens; pos_func).
//
// Same algebra as the tuned kernels, on raw weights: per head
//   q = Wq x,  u = Wkᵀ q / √E,  s_j = u · X0_j,  p = softmax(s),
//   z = Σ_j p_j X0_j,  v = Wv z,  a = U [v_h] + b_U
// (= the reference's (Wq x/e^¼)·(Wk k_j/e^¼) scores and Σ_j p_j Wv k_j values),
// so no per-token key / value is materialised.  Only the query rows the output
// needs are propagated (agent: token 0; mixer: the last A+3 tokens).
//
// Execution: one wave per query row (agent: one sequence; mixer: one workgroup
// per episode, its waves sharing the key block X0 in LDS).  Lane = feature for
// E-vectors; an H·E vector keeps head h in slot h, an FF vector element
// lane + 64 i in slot i.  Matrix-vector products broadcast their input through
// a per-wave LDS vector and read weights coalesced (the pack holds transposed
// copies, t2o_layout.hpp GenOffsets).  All arithmetic is fp32.  Weight grads:
// the big matrices through a record tape (GenRec) contracted by a tiled
// split-K GEMM (dW = Σ_records dY ⊗ X); vectors and the small embedding / head
// matrices in per-lane registers, flushed once per wave with float atomics.
// Gradients land in ONE slab in reference parameter order (unpack = add).
#include <math.h>

#include "t2o_common.hpp"
#include "t2o_generic.hpp"
#include "t2o_layout.hpp"

namespace t2o {
namespace {

constexpr int NSLOT = 8;    // per-lane slots of an HE- or FF-vector (HE <= 512, FF <= 512)
constexpr int TSLOT = 3;    // per-lane token slots (tokens <= 192)
constexpr int GMAXF = 16;   // entity / state features
constexpr int GMAXNA = 16;  // agent actions
constexpr int GVB = 512;    // per-wave broadcast vector
constexpr int GMAXD = T2O_MAX_DEPTH;

T2O_DEV int ln() { return threadIdx.x & 63; }

// make this wave's LDS writes visible to its own later reads (lanes exchange data)
T2O_DEV void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
T2O_DEV float wsum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
T2O_DEV float wmax(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// One network: dims and its generic pack
struct GNet {
  const float* w;
  GenOffsets g;
  int E, H, D, FF, F, NA;
  float scale;  // 1 / √E
};

T2O_DEV GNet make_net(const t2o_layout& L, const GenOffsets& g, const float* pack) {
  GNet n;
  n.w = pack;
  n.g = g;
  n.E = L.E;
  n.H = L.H;
  n.D = L.D;
  n.FF = L.FF;
  n.F = L.F;
  n.NA = L.NA;
  n.scale = 1.0f / sqrtf((float)L.E);
  return n;
}

// Per-wave LDS scratch
struct Scratch {
  float* vb;   // broadcast vector [GVB]
  float* vb2;  // second broadcast vector [GVB]
  float* pb;   // softmax probabilities of the block's heads [H][Lt]
  float* pb2;  // softmax backward scratch [Lt]
};
constexpr int scratch_floats(int H, int Lt) { return 2 * GVB + H * Lt + Lt; }
T2O_DEV Scratch make_scratch(float* base, int H, int Lt) {
  return Scratch{base, base + GVB, base + 2 * GVB, base + 2 * GVB + H * Lt};
}

// out[s] = Σ_{k < NI} M[k·ld + idx_s] · vin[k],  idx_s = s·S + lane (valid when
// lane < W and idx_s < NO): vin broadcast from LDS, M rows read coalesced
template <int NS>
T2O_DEV void gemv(const float* __restrict__ M, int64_t ld, const float* vin, int NI, int S, int W, int NO,
                  float (&out)[NS]) {
  const int l = ln();
  int idx[NS];
  bool ok[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    idx[s] = s * S + l;
    ok[s] = l < W && idx[s] < NO;
    out[s] = 0.f;
  }
#pragma unroll 2
  for (int k = 0; k < NI; ++k) {
    const float x = vin[k];
    const float* row = M + (int64_t)k * ld;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (ok[s]) out[s] = fmaf(row[idx[s]], x, out[s]);
  }
}
T2O_DEV float gemv1(const float* __restrict__ M, int64_t ld, const float* vin, int NI, int NO) {
  float o[1];
  gemv<1>(M, ld, vin, NI, 64, 64, NO, o);
  return o[0];
}

// vb <- E-vector / HE-vector (slots = heads) / FF-vector (slots of 64)
T2O_DEV void put_e(float* vb, float v, int E) {
  wsync();
  if (ln() < E) vb[ln()] = v;
  wsync();
}
T2O_DEV void put_he(float* vb, const float (&v)[NSLOT], int H, int E) {
  wsync();
  if (ln() < E)
    for (int h = 0; h < H; ++h) vb[h * E + ln()] = v[h];
  wsync();
}
T2O_DEV void put_ff(float* vb, const float (&v)[NSLOT], int FF, bool relu) {
  wsync();
#pragma unroll
  for (int i = 0; i < NSLOT; ++i) {
    const int k = ln() + 64 * i;
    if (k < FF) vb[k] = relu ? fmaxf(v[i], 0.f) : v[i];
  }
  wsync();
}

// LayerNorm over E lanes (eps 1e-5, biased variance)
T2O_DEV float ln_fwd(float r, int E, float gam, float bet, float& xh, float& rs) {
  const bool fe = ln() < E;
  const float mean = wsum(fe ? r : 0.f) / (float)E;
  const float dv = fe ? r - mean : 0.f;
  const float var = wsum(dv * dv) / (float)E;
  rs = 1.0f / sqrtf(var + 1e-5f);
  xh = dv * rs;
  return fe ? xh * gam + bet : 0.f;
}
T2O_DEV float ln_bwd(float gout, float xh, float rs, float gam, int E) {
  const bool fe = ln() < E;
  const float gx = fe ? gout * gam : 0.f;
  const float m1 = wsum(gx) / (float)E, m2 = wsum(gx * xh) / (float)E;
  return fe ? (gx - m1 - xh * m2) * rs : 0.f;
}

T2O_DEV float vget(const float* w, int64_t off, int n) { return ln() < n ? w[off + ln()] : 0.f; }

// ---- one transformer block for one query row --------------------------------
struct BCache {
  float x;                                   // block input
  float q[NSLOT], u[NSLOT], z[NSLOT], v[NSLOT];  // per head
  float xh1, rs1, y;
  float f1[NSLOT];                           // FFN pre-activation
  float xh2, rs2;
};

// X0: the layer-0 tokens [Lt][XS] (LDS).  Returns the block output; the heads'
// softmax probabilities stay in sc.pb for the backward.
T2O_DEV float block_fwd(const GNet& N, int d, const float* X0, int Lt, int XS, float x, BCache& c,
                        const Scratch& sc) {
  const int l = ln(), E = N.E, H = N.H, FF = N.FF, HE = H * E;
  const bool fe = l < E;
  const ParamOffsets& P = N.g.P;
  c.x = x;
  put_e(sc.vb, x, E);
  gemv<NSLOT>(N.w + N.g.WqT[d], HE, sc.vb, E, E, E, HE, c.q);  // q = Wq x
  for (int h = 0; h < H; ++h) {
    put_e(sc.vb2, c.q[h], E);
    c.u[h] = N.scale * gemv1(N.w + P.Wk[d] + (int64_t)h * E * E, E, sc.vb2, E, E);  // u = Wkᵀ q / √E
    put_e(sc.vb2, c.u[h], E);
    float s[TSLOT], m = -INFINITY;
#pragma unroll
    for (int mm = 0; mm < TSLOT; ++mm) {
      const int j = l + 64 * mm;
      s[mm] = -INFINITY;
      if (j < Lt) {
        float acc = 0.f;
        for (int f = 0; f < E; ++f) acc = fmaf(X0[j * XS + f], sc.vb2[f], acc);
        s[mm] = acc;
      }
      m = fmaxf(m, s[mm]);
    }
    m = wmax(m);
    float sum = 0.f;
#pragma unroll
    for (int mm = 0; mm < TSLOT; ++mm) {
      s[mm] = (l + 64 * mm < Lt) ? expf(s[mm] - m) : 0.f;
      sum += s[mm];
    }
    const float inv = 1.0f / wsum(sum);
    float* pbh = sc.pb + h * Lt;
#pragma unroll
    for (int mm = 0; mm < TSLOT; ++mm)
      if (l + 64 * mm < Lt) pbh[l + 64 * mm] = s[mm] * inv;
    wsync();
    float z = 0.f;
    if (fe)
      for (int j = 0; j < Lt; ++j) z = fmaf(pbh[j], X0[j * XS + l], z);
    c.z[h] = z;
  }
  for (int h = 0; h < H; ++h) {
    put_e(sc.vb2, c.z[h], E);
    c.v[h] = gemv1(N.w + N.g.WvT[d] + h * E, HE, sc.vb2, E, E);  // v = Wv z
  }
  put_he(sc.vb, c.v, H, E);
  const float a = gemv1(N.w + N.g.UT[d], E, sc.vb, HE, E);  // a = U v
  const float r1 = fe ? a + N.w[P.bu[d] + l] + x : 0.f;
  c.y = ln_fwd(r1, E, vget(N.w, P.g1[d], E), vget(N.w, P.n1[d], E), c.xh1, c.rs1);
  put_e(sc.vb, c.y, E);
  gemv<NSLOT>(N.w + N.g.W1T[d], FF, sc.vb, E, 64, 64, FF, c.f1);  // f1 = W1 y + c1
#pragma unroll
  for (int i = 0; i < NSLOT; ++i) {
    const int k = l + 64 * i;
    if (k < FF) c.f1[i] += N.w[P.c1[d] + k];
  }
  put_ff(sc.vb, c.f1, FF, true);
  float r2 = gemv1(N.w + N.g.W2T[d], E, sc.vb, FF, E);  // r2 = W2 relu(f1) + c2 + y
  r2 = fe ? r2 + N.w[P.c2[d] + l] + c.y : 0.f;
  return ln_fwd(r2, E, vget(N.w, P.g2[d], E), vget(N.w, P.n2[d], E), c.xh2, c.rs2);
}

// per-lane vector-grad partial sums of one block
struct VAcc {
  float bu, g1, n1, c2, g2, n2;
  float c1[NSLOT];
};
T2O_DEV void vacc_zero(VAcc& a) {
  a.bu = a.g1 = a.n1 = a.c2 = a.g2 = a.n2 = 0.f;
#pragma unroll
  for (int i = 0; i < NSLOT; ++i) a.c1[i] = 0.f;
}

// Backward of block_fwd (same X0, cache and sc.pb).  gx: grad wrt the block
// output; returns the grad wrt the block's query input.  Key-token grads are
// added into GX (LDS, [Lt][XS]; atomically when waves share it).  rec: this
// (row, step, block)'s tape record or null.
T2O_DEV float block_bwd(const GNet& N, int d, const float* X0, float* GX, bool gx_atomic, int Lt, int XS,
                        const BCache& c, float gx, VAcc& va, float* rec, const GenRec& R, const Scratch& sc) {
  const int l = ln(), E = N.E, H = N.H, FF = N.FF, HE = H * E;
  const bool fe = l < E;
  const ParamOffsets& P = N.g.P;
  gx = fe ? gx : 0.f;
  va.g2 += gx * c.xh2;
  va.n2 += gx;
  const float gr2 = ln_bwd(gx, c.xh2, c.rs2, vget(N.w, P.g2[d], E), E);
  va.c2 += gr2;
  put_e(sc.vb, gr2, E);
  float gf1[NSLOT];
  gemv<NSLOT>(N.w + P.W2[d], FF, sc.vb, E, 64, 64, FF, gf1);  // W2ᵀ gr2
#pragma unroll
  for (int i = 0; i < NSLOT; ++i) {
    gf1[i] = c.f1[i] > 0.f ? gf1[i] : 0.f;
    va.c1[i] += gf1[i];
  }
  if (rec) {
    if (fe) {
      rec[R.GR2 + l] = gr2;
      rec[R.Y + l] = c.y;
    }
#pragma unroll
    for (int i = 0; i < NSLOT; ++i) {
      const int k = l + 64 * i;
      if (k < FF) {
        rec[R.FR + k] = fmaxf(c.f1[i], 0.f);
        rec[R.GF1 + k] = gf1[i];
      }
    }
  }
  put_ff(sc.vb, gf1, FF, false);
  float gy = gemv1(N.w + P.W1[d], E, sc.vb, FF, E) + gr2;  // W1ᵀ gf1 + residual
  gy = fe ? gy : 0.f;
  va.g1 += gy * c.xh1;
  va.n1 += gy;
  const float ga = ln_bwd(gy, c.xh1, c.rs1, vget(N.w, P.g1[d], E), E);
  va.bu += ga;
  float gxq = ga;  // the LN1 residual: grad wrt the query input
  put_e(sc.vb, ga, E);
  float gv[NSLOT];
  gemv<NSLOT>(N.w + P.U[d], HE, sc.vb, E, E, E, HE, gv);  // Uᵀ ga
  if (rec && fe) {
    rec[R.GA + l] = ga;
    for (int h = 0; h < H; ++h) rec[R.V + h * E + l] = c.v[h];
  }
  for (int h = 0; h < H; ++h) {
    put_e(sc.vb2, gv[h], E);
    const float gz = gemv1(N.w + P.Wv[d] + (int64_t)h * E * E, E, sc.vb2, E, E);  // Wv_hᵀ gv_h
    if (rec && fe) {
      rec[R.GV + h * E + l] = gv[h];
      rec[R.Z + h * E + l] = c.z[h];
    }
    // softmax backward: gp_j = gz · X0_j, gs_j = p_j (gp_j - Σ p gp)
    put_e(sc.vb2, gz, E);
    const float* pbh = sc.pb + h * Lt;
    float gp[TSLOT], dot = 0.f;
#pragma unroll
    for (int mm = 0; mm < TSLOT; ++mm) {
      const int j = l + 64 * mm;
      gp[mm] = 0.f;
      if (j < Lt) {
        float acc = 0.f;
        for (int f = 0; f < E; ++f) acc = fmaf(X0[j * XS + f], sc.vb2[f], acc);
        gp[mm] = acc;
        dot += pbh[j] * acc;
      }
    }
    dot = wsum(dot);
#pragma unroll
    for (int mm = 0; mm < TSLOT; ++mm) {
      const int j = l + 64 * mm;
      if (j < Lt) sc.pb2[j] = pbh[j] * (gp[mm] - dot);
    }
    wsync();
    // gu = Σ_j gs_j X0_j;  GX_j += p_j gz + gs_j u
    float gu = 0.f;
    if (fe) {
      const float uh = c.u[h];
      for (int j = 0; j < Lt; ++j) {
        const float gs = sc.pb2[j];
        gu = fmaf(gs, X0[j * XS + l], gu);
        const float add = pbh[j] * gz + gs * uh;
        if (gx_atomic) atomicAdd(GX + j * XS + l, add);
        else GX[j * XS + l] += add;
      }
    }
    put_e(sc.vb2, gu, E);
    const float gq = N.scale * gemv1(N.w + N.g.WkT[d] + h * E, HE, sc.vb2, E, E);  // Wk_h gu / √E
    if (rec && fe) {
      rec[R.Q + h * E + l] = c.q[h];
      rec[R.GU + h * E + l] = N.scale * gu;
      rec[R.GQ + h * E + l] = gq;
    }
    put_e(sc.vb2, gq, E);
    gxq += gemv1(N.w + P.Wq[d] + (int64_t)h * E * E, E, sc.vb2, E, E);  // Wq_hᵀ gq_h
  }
  if (rec && fe) rec[R.X + l] = c.x;
  return fe ? gxq : 0.f;
}

// flush one wave's block-vector partial sums into the (reference-order) slab
T2O_DEV void vacc_flush(const GNet& N, float* gs, int d, const VAcc& a) {
  const int l = ln(), E = N.E;
  const ParamOffsets& P = N.g.P;
  if (l < E) {
    unsafeAtomicAdd(gs + P.bu[d] + l, a.bu);
    unsafeAtomicAdd(gs + P.g1[d] + l, a.g1);
    unsafeAtomicAdd(gs + P.n1[d] + l, a.n1);
    unsafeAtomicAdd(gs + P.c2[d] + l, a.c2);
    unsafeAtomicAdd(gs + P.g2[d] + l, a.g2);
    unsafeAtomicAdd(gs + P.n2[d] + l, a.n2);
  }
#pragma unroll
  for (int i = 0; i < NSLOT; ++i) {
    const int k = l + 64 * i;
    if (k < N.FF) unsafeAtomicAdd(gs + P.c1[d] + k, a.c1[i]);
  }
}

// ============================================================================
// Agent
// ============================================================================
struct GAgentNet {
  const float* pack;
  const float* h0;
  float* q;
  float* h;
  float* hmid;
};

struct GAgentArgs {
  t2o_layout L;
  GenOffsets g;
  GenRec R;
  GAgentNet net[2];
  const float* obs;
  int64_t obs_sb, obs_st;
  // backward
  const float* h0;
  const float* h_seq;
  const float* hmid;
  int h_ts;
  const float* gq;
  const float* gchosen;
  const int64_t* actions;
  int64_t act_sb, act_st;
  const float* gh;
  float* slab;
  float* tape;
  float* gh0;
  int B, T, A, waves, XS, Lt;
  int64_t rpad;  // rows per step in the tape (16-row tiles)
};

__host__ __device__ inline int agent_wave_floats(int Lt, int XS, int n, int F, int H) {
  return 2 * Lt * XS + n * F + scratch_floats(H, Lt);
}

// X0 = [h; We o_j + be] of one row's step; the observations to OB [n][F]
T2O_DEV void agent_tokens(const GNet& N, const float* __restrict__ ob, int n, float h, float* X0, int XS,
                          float* OB) {
  const int l = ln(), E = N.E, F = N.F;
  wsync();
  for (int i = l; i < n * F; i += 64) OB[i] = ob[i];
  if (l < E) X0[l] = h;
  wsync();
  if (l < E) {
    const float be = N.w[N.g.P.be + l];
    for (int j = 0; j < n; ++j) {
      float acc = be;
      for (int i = 0; i < F; ++i) acc = fmaf(N.w[N.g.WeT + i * E + l], OB[j * F + i], acc);
      X0[(j + 1) * XS + l] = acc;
    }
  }
  wsync();
}

__global__ __launch_bounds__(256) void gagent_fwd_kernel(GAgentArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const t2o_layout& L = a.L;
  const GAgentNet net = a.net[blockIdx.y];
  const GNet N = make_net(L, a.g, net.pack);
  const int w = threadIdx.x >> 6, l = ln();
  const int R = a.B * a.A, n = L.n_ent, E = N.E, Lt = a.Lt, XS = a.XS;
  const int row = blockIdx.x * a.waves + w;
  if (row >= R) return;  // wave-uniform; no block barriers below
  float* X0 = smem + (size_t)w * agent_wave_floats(Lt, XS, n, N.F, N.H);
  float* OB = X0 + 2 * Lt * XS;
  const Scratch sc = make_scratch(OB + n * N.F, N.H, Lt);
  const int b = row / a.A, ag = row % a.A;
  const bool fe = l < E;
  float x = (net.h0 && fe) ? net.h0[(size_t)row * E + l] : 0.f;
  for (int t = 0; t < a.T; ++t) {
    agent_tokens(N, a.obs + b * a.obs_sb + t * a.obs_st + (int64_t)ag * n * N.F, n, x, X0, XS, OB);
    for (int d = 0; d < N.D; ++d) {
      if (d > 0 && net.hmid && fe) net.hmid[((((size_t)b * a.T + t) * (N.D - 1) + d - 1) * a.A + ag) * E + l] = x;
      BCache c;
      x = block_fwd(N, d, X0, Lt, XS, x, c, sc);
    }
    put_e(sc.vb, x, E);
    const size_t base = ((size_t)b * a.T + t) * a.A + ag;
    if (l < N.NA) {
      float qv = N.w[N.g.P.bo + l];
      for (int f = 0; f < E; ++f) qv = fmaf(N.w[N.g.WoT + f * N.NA + l], sc.vb[f], qv);
      net.q[base * N.NA + l] = qv;
    }
    if (fe) net.h[base * E + l] = x;
  }
}

__global__ __launch_bounds__(256) void gagent_bwd_kernel(GAgentArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const t2o_layout& L = a.L;
  const GNet N = make_net(L, a.g, a.net[0].pack);
  const int w = threadIdx.x >> 6, l = ln();
  const int R = a.B * a.A, n = L.n_ent, E = N.E, F = N.F, NA = N.NA, Lt = a.Lt, XS = a.XS;
  const int row = blockIdx.x * a.waves + w;
  if (row >= R) return;
  float* X0 = smem + (size_t)w * agent_wave_floats(Lt, XS, n, F, N.H);
  float* GX = X0 + Lt * XS;
  float* OB = GX + Lt * XS;
  const Scratch sc = make_scratch(OB + n * F, N.H, Lt);
  const int b = row / a.A, ag = row % a.A;
  const bool fe = l < E;
  const ParamOffsets& P = N.g.P;
  VAcc va[GMAXD];
  for (int d = 0; d < GMAXD; ++d) vacc_zero(va[d]);
  float gWe[GMAXF], gWo[GMAXNA], gbe = 0.f, gbo = 0.f;
#pragma unroll
  for (int i = 0; i < GMAXF; ++i) gWe[i] = 0.f;
#pragma unroll
  for (int i = 0; i < GMAXNA; ++i) gWo[i] = 0.f;
  float grec = 0.f;  // dL/dh_t from step t+1
  const size_t DT = (size_t)a.T * a.rpad;  // records per block
  for (int t = a.T - 1; t >= 0; --t) {
    float hp = 0.f;
    if (t > 0) hp = fe ? a.h_seq[(((size_t)b * a.h_ts + t - 1) * a.A + ag) * E + l] : 0.f;
    else if (a.h0 && fe) hp = a.h0[(size_t)row * E + l];
    agent_tokens(N, a.obs + b * a.obs_sb + t * a.obs_st + (int64_t)ag * n * F, n, hp, X0, XS, OB);
    for (int i = l; i < Lt * XS; i += 64) GX[i] = 0.f;
    const size_t sidx = ((size_t)b * a.T + t) * a.A + ag;
    float gx = grec + ((a.gh && fe) ? a.gh[sidx * E + l] : 0.f);
    // head q = Wo x_D + bo (x_D = h_t, the forward output)
    float gq = 0.f;
    if (l < NA) {
      if (a.gq) gq = a.gq[sidx * NA + l];
      if (a.gchosen && a.actions[b * a.act_sb + t * a.act_st + ag] == l) gq += a.gchosen[sidx];
    }
    gbo += gq;
    const float xD = fe ? a.h_seq[(((size_t)b * a.h_ts + t) * a.A + ag) * E + l] : 0.f;
    wsync();
    if (l < NA) sc.vb2[l] = gq;
    wsync();
    if (fe) {
#pragma unroll
      for (int k = 0; k < GMAXNA; ++k)
        if (k < NA) {
          gWo[k] += sc.vb2[k] * xD;
          gx = fmaf(N.w[P.Wo + k * E + l], sc.vb2[k], gx);
        }
    }
    for (int d = N.D - 1; d >= 0; --d) {
      float xin = hp;
      if (d > 0) {
        if (a.hmid) {
          xin = fe ? a.hmid[((((size_t)b * a.h_ts + t) * (N.D - 1) + d - 1) * a.A + ag) * E + l] : 0.f;
        } else {
          for (int dd = 0; dd < d; ++dd) {
            BCache c0;
            xin = block_fwd(N, dd, X0, Lt, XS, xin, c0, sc);
          }
        }
      }
      BCache c;
      (void)block_fwd(N, d, X0, Lt, XS, xin, c, sc);
      float* rec = a.tape + ((size_t)d * DT + (size_t)t * a.rpad + row) * a.R.SIZE;
      gx = block_bwd(N, d, X0, GX, false, Lt, XS, c, gx, va[d], rec, a.R, sc);
    }
    wsync();
    // grad wrt h_{t-1}: the query path plus token 0's key path
    grec = fe ? gx + GX[l] : 0.f;
    // entity tokens: embedding grads
    if (fe) {
      for (int j = 0; j < n; ++j) {
        const float g = GX[(j + 1) * XS + l];
        gbe += g;
#pragma unroll
        for (int i = 0; i < GMAXF; ++i)
          if (i < F) gWe[i] = fmaf(g, OB[j * F + i], gWe[i]);
      }
    }
  }
  if (a.gh0 && fe) a.gh0[(size_t)row * E + l] = grec;
  float* gs = a.slab;
  for (int d = 0; d < N.D; ++d) vacc_flush(N, gs, d, va[d]);
  if (fe) {
    unsafeAtomicAdd(gs + P.be + l, gbe);
#pragma unroll
    for (int i = 0; i < GMAXF; ++i)
      if (i < F) unsafeAtomicAdd(gs + P.We + l * F + i, gWe[i]);
#pragma unroll
    for (int k = 0; k < GMAXNA; ++k)
      if (k < NA) unsafeAtomicAdd(gs + P.Wo + k * E + l, gWo[k]);
  }
  if (l < NA) unsafeAtomicAdd(gs + P.bo + l, gbo);
}

// ============================================================================
// Mixer
// ============================================================================
struct GMixNet {
  const float* pack;
  const float* hw0;
  const float* hid;
  const float* qsel;   // qmode 1/2: [b][q_ts][a][NA]
  const float* qv_in;  // qmode 0: [B][T][A]
  int qmode, T;
  float* y;
  float* hw;
  float* qv;
  float* xout;
  float* xmid;
};

struct GMixArgs {
  t2o_layout L;
  GenOffsets g;
  GenRec R;
  GMixNet net[2];
  const float* states;
  int64_t st_sb, st_st;
  int64_t hid_sb, hid_st;
  const float* qarg;
  int q_ts, n_actions;
  const int64_t* actions;
  int64_t act_sb, act_st;
  const int32_t* avail;
  int64_t av_sb, av_st;
  // backward
  const float* hw;
  const float* xout;
  const float* xmid;
  const float* gy;
  const float* ghw_ext;
  float* gqv;
  float* ghid;
  float* ghw0;
  float* slab;
  float* tape;
  int B, waves, XS, Lt, ns, A, Q, qpad;
};

// shared LDS of a mixer workgroup, then per-wave scratch
struct MixLds {
  float *X0, *GX, *OUT, *GOUT, *ST, *QV, *GHW, *waves;
};
T2O_DEV MixLds mix_lds(float* s, int Lt, int XS, int Q, int E, int ns, int Fs, int A) {
  MixLds m;
  m.X0 = s;
  m.GX = m.X0 + Lt * XS;
  m.OUT = m.GX + Lt * XS;
  m.GOUT = m.OUT + Q * E;
  m.ST = m.GOUT + Q * E;
  m.QV = m.ST + ((ns * Fs + 3) / 4) * 4;
  m.GHW = m.QV + ((A + 3) / 4) * 4;
  m.waves = m.GHW + 3 * E;
  return m;
}
inline size_t mix_lds_floats(int Lt, int XS, int Q, int E, int ns, int Fs, int A, int H, int waves) {
  return (size_t)2 * Lt * XS + 2 * Q * E + ((ns * Fs + 3) / 4) * 4 + ((A + 3) / 4) * 4 + 3 * E +
         (size_t)waves * scratch_floats(H, Lt);
}

T2O_DEV float elu1(float x) { return x > 0.f ? x : expm1f(x); }

// state-token embeddings (rows 0..ns-1 of X0) from ST, by the whole workgroup
T2O_DEV void mix_embed(const GNet& N, const MixLds& m, int ns, int XS) {
  const int E = N.E, F = N.F;
  for (int i = threadIdx.x; i < ns * E; i += blockDim.x) {
    const int j = i / E, f = i % E;
    float acc = N.w[N.g.P.be + f];
    for (int k = 0; k < F; ++k) acc = fmaf(N.w[N.g.P.We + f * F + k], m.ST[j * F + k], acc);
    m.X0[j * XS + f] = acc;
  }
}

__global__ __launch_bounds__(256) void gmixer_fwd_kernel(GMixArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const t2o_layout& L = a.L;
  const GMixNet net = a.net[blockIdx.y];
  const GNet N = make_net(L, a.g, net.pack);
  const int E = N.E, H = N.H, F = N.F, Lt = a.Lt, XS = a.XS, ns = a.ns, A = a.A, Q = a.Q;
  const int b = blockIdx.x, w = threadIdx.x >> 6, l = ln(), tid = threadIdx.x, nt = blockDim.x;
  const MixLds m = mix_lds(smem, Lt, XS, Q, E, ns, F, A);
  const Scratch sc = make_scratch(m.waves + (size_t)w * scratch_floats(H, Lt), H, Lt);
  const bool fe = l < E;
  for (int i = tid; i < 3 * E; i += nt) m.X0[(ns + A + i / E) * XS + i % E] = net.hw0 ? net.hw0[(size_t)b * 3 * E + i] : 0.f;
  for (int t = 0; t < net.T; ++t) {
    const float* st = a.states + b * a.st_sb + t * a.st_st;
    for (int i = tid; i < ns * F; i += nt) m.ST[i] = st[i];
    const float* hd = net.hid + b * a.hid_sb + t * a.hid_st;
    for (int i = tid; i < A * E; i += nt) m.X0[(ns + i / E) * XS + i % E] = hd[i];
    if (tid < A) {  // this agent's mixer input: qvals, chosen Q, or double-Q
      float qv;
      const int NA = a.n_actions;
      if (net.qmode == 0) {
        qv = net.qv_in[((size_t)b * net.T + t) * A + tid];
      } else {
        const size_t qrow = (((size_t)b * a.q_ts + t) * A + tid) * NA;
        int act = 0;
        if (net.qmode == 1) {
          act = (int)a.actions[b * a.act_sb + t * a.act_st + tid];
        } else {
          const int32_t* av = a.avail ? a.avail + b * a.av_sb + t * a.av_st + tid * NA : nullptr;
          float best = -INFINITY;
          for (int k = 0; k < NA; ++k) {
            const float v = (av && av[k] == 0) ? -9999999.0f : a.qarg[qrow + k];
            if (k == 0 || v > best) {
              best = v;
              act = k;
            }
          }
        }
        qv = net.qsel[qrow + act];
      }
      m.QV[tid] = qv;
      if (net.qv) net.qv[((size_t)b * net.T + t) * A + tid] = qv;
    }
    __syncthreads();
    mix_embed(N, m, ns, XS);
    __syncthreads();
    for (int r = w; r < Q; r += a.waves) {
      float x = fe ? m.X0[(ns + r) * XS + l] : 0.f;
      for (int d = 0; d < N.D; ++d) {
        if (d > 0 && net.xmid && fe) net.xmid[((((size_t)b * net.T + t) * (N.D - 1) + d - 1) * Q + r) * E + l] = x;
        BCache c;
        x = block_fwd(N, d, m.X0, Lt, XS, x, c, sc);
      }
      if (fe) m.OUT[r * E + l] = x;
    }
    __syncthreads();
    const size_t bt = (size_t)b * net.T + t;
    if (w == 0) {  // mixing head (n_transf_mixer.py:75-89), lane = feature
      float ph = fe ? m.OUT[A * E + l] : 0.f;
      for (int ag = 0; ag < A; ++ag) ph += fe ? m.QV[ag] * posf(m.OUT[ag * E + l], L.pos_func, L.pos_beta) : 0.f;
      const float hidden = elu1(ph);
      const float w2 = fe ? posf(m.OUT[(A + 1) * E + l], L.pos_func, L.pos_beta) : 0.f;
      const float yv = wsum(fe ? hidden * w2 : 0.f);
      const float p2 = wsum(fe ? N.w[N.g.P.Wo + l] * m.OUT[(A + 2) * E + l] : 0.f) + N.w[N.g.P.bo];
      if (l == 0) net.y[bt] = yv + fmaxf(p2, 0.f);
    }
    for (int i = tid; i < 3 * E; i += nt) net.hw[bt * 3 * E + i] = m.OUT[A * E + i];
    if (net.xout)
      for (int i = tid; i < Q * E; i += nt) net.xout[bt * Q * E + i] = m.OUT[i];
    __syncthreads();
    for (int i = tid; i < 3 * E; i += nt) m.X0[(ns + A + i / E) * XS + i % E] = m.OUT[A * E + i];
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void gmixer_bwd_kernel(GMixArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const t2o_layout& L = a.L;
  const GMixNet& net = a.net[0];
  const GNet N = make_net(L, a.g, net.pack);
  const int E = N.E, H = N.H, F = N.F, Lt = a.Lt, XS = a.XS, ns = a.ns, A = a.A, Q = a.Q, T = net.T;
  const int b = blockIdx.x, w = threadIdx.x >> 6, l = ln(), tid = threadIdx.x, nt = blockDim.x;
  const MixLds m = mix_lds(smem, Lt, XS, Q, E, ns, F, A);
  const Scratch sc = make_scratch(m.waves + (size_t)w * scratch_floats(H, Lt), H, Lt);
  const bool fe = l < E;
  const ParamOffsets& P = N.g.P;
  VAcc va[GMAXD];
  for (int d = 0; d < GMAXD; ++d) vacc_zero(va[d]);
  float gWe[GMAXF], gbe = 0.f, gWo = 0.f, gbo = 0.f;
#pragma unroll
  for (int i = 0; i < GMAXF; ++i) gWe[i] = 0.f;
  for (int i = tid; i < 3 * E; i += nt) m.GHW[i] = 0.f;
  const size_t DT = (size_t)T * a.B * a.qpad;  // records per block
  for (int t = T - 1; t >= 0; --t) {
    const size_t bt = (size_t)b * T + t;
    const float* st = a.states + b * a.st_sb + t * a.st_st;
    for (int i = tid; i < ns * F; i += nt) m.ST[i] = st[i];
    const float* hd = net.hid + b * a.hid_sb + t * a.hid_st;
    for (int i = tid; i < A * E; i += nt) m.X0[(ns + i / E) * XS + i % E] = hd[i];
    for (int i = tid; i < 3 * E; i += nt)
      m.X0[(ns + A + i / E) * XS + i % E] =
          t > 0 ? a.hw[(bt - 1) * 3 * E + i] : (net.hw0 ? net.hw0[(size_t)b * 3 * E + i] : 0.f);
    for (int i = tid; i < Q * E; i += nt) m.OUT[i] = a.xout[bt * Q * E + i];
    for (int i = tid; i < A; i += nt) m.QV[i] = net.qv_in[bt * A + i];
    for (int i = tid; i < Lt * XS; i += nt) m.GX[i] = 0.f;
    __syncthreads();
    mix_embed(N, m, ns, XS);
    if (w == 0) {  // mixing-head backward, lane = feature
      const float gyv = a.gy[bt];
      float ph = fe ? m.OUT[A * E + l] : 0.f;
      for (int ag = 0; ag < A; ++ag) ph += fe ? m.QV[ag] * posf(m.OUT[ag * E + l], L.pos_func, L.pos_beta) : 0.f;
      const float hidden = elu1(ph);
      const float x2raw = fe ? m.OUT[(A + 1) * E + l] : 0.f;
      const float w2 = fe ? posf(x2raw, L.pos_func, L.pos_beta) : 0.f;
      const float x3 = fe ? m.OUT[(A + 2) * E + l] : 0.f;
      const float wo = fe ? N.w[P.Wo + l] : 0.f;
      const float p2 = wsum(wo * x3) + N.w[P.bo];
      const float gph = fe ? gyv * w2 * (ph > 0.f ? 1.f : expf(ph)) : 0.f;
      const float gp2 = p2 > 0.f ? gyv : 0.f;
      for (int ag = 0; ag < A; ++ag) {
        const float xa = fe ? m.OUT[ag * E + l] : 0.f;
        const float gq = wsum(fe ? gph * posf(xa, L.pos_func, L.pos_beta) : 0.f);
        if (l == 0) a.gqv[bt * A + ag] = gq;
        if (fe) m.GOUT[ag * E + l] = gph * m.QV[ag] * dposf(xa, L.pos_func, L.pos_beta);
      }
      if (fe) {
        const float* gx = a.ghw_ext ? a.ghw_ext + bt * 3 * E : nullptr;
        m.GOUT[A * E + l] = gph + m.GHW[l] + (gx ? gx[l] : 0.f);
        m.GOUT[(A + 1) * E + l] =
            gyv * hidden * dposf(x2raw, L.pos_func, L.pos_beta) + m.GHW[E + l] + (gx ? gx[E + l] : 0.f);
        m.GOUT[(A + 2) * E + l] = gp2 * wo + m.GHW[2 * E + l] + (gx ? gx[2 * E + l] : 0.f);
        gWo += gp2 * x3;
      }
      if (l == 0) gbo += gp2;
    }
    __syncthreads();
    for (int r = w; r < Q; r += a.waves) {
      float gx = fe ? m.GOUT[r * E + l] : 0.f;
      for (int d = N.D - 1; d >= 0; --d) {
        float xin = fe ? m.X0[(ns + r) * XS + l] : 0.f;
        if (d > 0) {
          if (a.xmid) {
            xin = fe ? a.xmid[(((bt * (N.D - 1)) + d - 1) * Q + r) * E + l] : 0.f;
          } else {
            for (int dd = 0; dd < d; ++dd) {
              BCache c0;
              xin = block_fwd(N, dd, m.X0, Lt, XS, xin, c0, sc);
            }
          }
        }
        BCache c;
        (void)block_fwd(N, d, m.X0, Lt, XS, xin, c, sc);
        float* rec = a.tape + ((size_t)d * DT + ((size_t)t * a.B + b) * a.qpad + r) * a.R.SIZE;
        gx = block_bwd(N, d, m.X0, m.GX, true, Lt, XS, c, gx, va[d], rec, a.R, sc);
      }
      if (fe) atomicAdd(m.GX + (ns + r) * XS + l, gx);  // the query path of block 0
    }
    __syncthreads();
    for (int i = tid; i < A * E; i += nt) a.ghid[bt * A * E + i] = m.GX[(ns + i / E) * XS + i % E];
    for (int i = tid; i < 3 * E; i += nt) m.GHW[i] = m.GX[(ns + A + i / E) * XS + i % E];
    if (fe) {  // state-token embedding grads, tokens dealt over the waves
      for (int j = w; j < ns; j += a.waves) {
        const float g = m.GX[j * XS + l];
        gbe += g;
#pragma unroll
        for (int k = 0; k < GMAXF; ++k)
          if (k < F) gWe[k] = fmaf(g, m.ST[j * F + k], gWe[k]);
      }
    }
    __syncthreads();
  }
  if (a.ghw0)
    for (int i = tid; i < 3 * E; i += nt) a.ghw0[(size_t)b * 3 * E + i] = m.GHW[i];
  float* gs = a.slab;
  for (int d = 0; d < N.D; ++d) vacc_flush(N, gs, d, va[d]);
  if (fe) {
    unsafeAtomicAdd(gs + P.be + l, gbe);
#pragma unroll
    for (int k = 0; k < GMAXF; ++k)
      if (k < F) unsafeAtomicAdd(gs + P.We + l * F + k, gWe[k]);
    if (w == 0) unsafeAtomicAdd(gs + P.Wo + l, gWo);
  }
  if (w == 0 && l == 0) unsafeAtomicAdd(gs + P.bo, gbo);
}

// ============================================================================
// Weight-gradient contraction: C[m][n] += Σ_k A_k[ao + m] · B_k[bo + n] over
// the tape's records k (row-major, SIZE floats each), batched over heads.
// ============================================================================
struct GemmTask {
  int M, N, batch, ldc;
  int ao, bo, a_bs, b_bs;
  int64_t co, c_bs;
};

constexpr int GT = 64, GK = 16;

__global__ __launch_bounds__(256) void ggemm_kernel(const float* __restrict__ rec, int64_t nrec, int S, GemmTask tk,
                                                    float* __restrict__ C, int64_t kchunk) {
  __shared__ float As[GK][GT + 4], Bs[GK][GT + 4];
  const int tiles_m = (tk.M + GT - 1) / GT;
  const int m0 = (blockIdx.x % tiles_m) * GT, n0 = (blockIdx.x / tiles_m) * GT, z = blockIdx.z;
  const int ao = tk.ao + z * tk.a_bs, bo = tk.bo + z * tk.b_bs;
  const int64_t k0 = (int64_t)blockIdx.y * kchunk;
  const int64_t k1 = k0 + kchunk < nrec ? k0 + kchunk : nrec;
  const int tid = threadIdx.x, tx = tid % 16, ty = tid / 16;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int64_t kb = k0; kb < k1; kb += GK) {
    for (int e = tid; e < GK * GT; e += 256) {
      const int kk = e / GT, c = e % GT;
      const int64_t r = kb + kk;
      const bool rok = r < k1;
      As[kk][c] = (rok && m0 + c < tk.M) ? rec[r * S + ao + m0 + c] : 0.f;
      Bs[kk][c] = (rok && n0 + c < tk.N) ? rec[r * S + bo + n0 + c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        av[i] = As[kk][ty * 4 + i];
        bv[i] = Bs[kk][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  if (k0 >= k1) return;
  float* Cz = C + tk.co + z * tk.c_bs;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int mm = m0 + ty * 4 + i, nn = n0 + tx * 4 + j;
      if (mm < tk.M && nn < tk.N) unsafeAtomicAdd(Cz + (int64_t)mm * tk.ldc + nn, acc[i][j]);
    }
}

int launch_gemm(const float* rec, int64_t nrec, int S, const GemmTask& tk, float* C, hipStream_t s) {
  const int tiles = ((tk.M + GT - 1) / GT) * ((tk.N + GT - 1) / GT);
  int64_t ksplit = 2048 / ((int64_t)tiles * tk.batch);
  if (ksplit < 1) ksplit = 1;
  const int64_t kmax = (nrec + 63) / 64;
  if (ksplit > kmax) ksplit = kmax > 0 ? kmax : 1;
  int64_t kchunk = (nrec + ksplit - 1) / ksplit;
  kchunk = (kchunk + GK - 1) / GK * GK;
  ksplit = (nrec + kchunk - 1) / kchunk;
  if (ksplit < 1) ksplit = 1;
  hipLaunchKernelGGL(ggemm_kernel, dim3(tiles, (unsigned)ksplit, tk.batch), dim3(256), 0, s, rec, nrec, S, tk, C, kchunk);
  return (int)hipGetLastError();
}

bool gen_limits(const t2o_layout& L) {
  return L.E >= 1 && L.E <= 64 && L.H >= 1 && L.H <= NSLOT && L.H * L.E <= GVB && L.D >= 1 && L.D <= GMAXD &&
         L.FF >= 1 && L.FF <= 64 * NSLOT && L.F >= 1 && L.F <= GMAXF && L.NA >= 1 && L.NA <= GMAXNA;
}

}  // namespace

// ---- entry points -----------------------------------------------------------
int64_t gen_tape_floats(const t2o_layout* L, int64_t tiles) {
  return (int64_t)L->D * tiles * 16 * gen_rec(L->E, L->H, L->FF).SIZE;
}

int gen_agent_unroll_fwd(const t2o_layout* L, const float* pack_on, const float* pack_tg, const float* obs,
                         int64_t obs_sb, int64_t obs_st, const float* h0_on, const float* h0_tg, float* q_on,
                         float* h_on, float* hmid_on, float* q_tg, float* h_tg, float* hmid_tg, int B, int T, int A,
                         hipStream_t stream) {
  if (!gen_limits(*L) || L->n_ent > 64) return T2O_EUNSUPPORTED;
  GAgentArgs a{};
  a.L = *L;
  a.g = gen_offsets(0, L->E, L->H, L->D, L->F, L->NA, L->FF);
  a.R = gen_rec(L->E, L->H, L->FF);
  a.net[0] = GAgentNet{pack_on, h0_on, q_on, h_on, hmid_on};
  int nnet = 1;
  if (pack_tg) {
    if (!q_tg || !h_tg) return T2O_EINVAL;
    a.net[1] = GAgentNet{pack_tg, h0_tg, q_tg, h_tg, hmid_tg};
    nnet = 2;
  }
  a.obs = obs;
  a.obs_sb = obs_sb;
  a.obs_st = obs_st;
  a.B = B;
  a.T = T;
  a.A = A;
  a.Lt = L->n_ent + 1;
  a.XS = L->E + 1;
  const size_t per = sizeof(float) * agent_wave_floats(a.Lt, a.XS, L->n_ent, L->F, L->H);
  a.waves = 4;
  while (a.waves > 1 && a.waves * per > 160 * 1024) a.waves >>= 1;
  if (a.waves * per > 160 * 1024) return T2O_EUNSUPPORTED;
  const size_t lds = a.waves * per;
  (void)hipFuncSetAttribute((const void*)gagent_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int R = B * A;
  hipLaunchKernelGGL(gagent_fwd_kernel, dim3((R + a.waves - 1) / a.waves, nnet), dim3(64 * a.waves), lds, stream, a);
  return (int)hipGetLastError();
}

int gen_agent_unroll_bwd(const t2o_layout* L, const float* pack, const float* obs, int64_t obs_sb, int64_t obs_st,
                         const float* h0, const float* h_seq, const float* hmid, int h_ts, const float* gq,
                         const float* gchosen, const int64_t* actions, int64_t act_sb, int64_t act_st,
                         const float* gh, float* gslabs, int max_slabs, int* nslab, void* tape, float* gh0, int B,
                         int T, int A, hipStream_t stream) {
  if (!gen_limits(*L) || L->n_ent > 64) return T2O_EUNSUPPORTED;
  if (max_slabs < 1) return T2O_EINVAL;
  GAgentArgs a{};
  a.L = *L;
  a.g = gen_offsets(0, L->E, L->H, L->D, L->F, L->NA, L->FF);
  a.R = gen_rec(L->E, L->H, L->FF);
  a.net[0] = GAgentNet{pack, nullptr, nullptr, nullptr, nullptr};
  a.obs = obs;
  a.obs_sb = obs_sb;
  a.obs_st = obs_st;
  a.h0 = h0;
  a.h_seq = h_seq;
  a.hmid = hmid;
  a.h_ts = h_ts;
  a.gq = gq;
  a.gchosen = gchosen;
  a.actions = actions;
  a.act_sb = act_sb;
  a.act_st = act_st;
  a.gh = gh;
  a.slab = gslabs;
  a.tape = static_cast<float*>(tape);
  a.gh0 = gh0;
  a.B = B;
  a.T = T;
  a.A = A;
  a.Lt = L->n_ent + 1;
  a.XS = L->E + 1;
  a.rpad = ((int64_t)B * A + 15) / 16 * 16;
  const int R = B * A;
  // one slab, reference parameter order; padding records of the tape stay zero
  hipError_t e = hipMemsetAsync(gslabs, 0, sizeof(float) * (size_t)L->grad_total, stream);
  if (e == hipSuccess)
    e = hipMemsetAsync(tape, 0, sizeof(float) * (size_t)gen_tape_floats(L, (int64_t)T * (a.rpad / 16)), stream);
  if (e != hipSuccess) return (int)e;
  const size_t per = sizeof(float) * agent_wave_floats(a.Lt, a.XS, L->n_ent, L->F, L->H);
  a.waves = 4;
  while (a.waves > 1 && a.waves * per > 160 * 1024) a.waves >>= 1;
  if (a.waves * per > 160 * 1024) return T2O_EUNSUPPORTED;
  const size_t lds = a.waves * per;
  (void)hipFuncSetAttribute((const void*)gagent_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(gagent_bwd_kernel, dim3((R + a.waves - 1) / a.waves), dim3(64 * a.waves), lds, stream, a);
  *nslab = 1;
  return (int)hipGetLastError();
}

static int mixer_launch_dims(const t2o_layout* L, GMixArgs& a, size_t& lds) {
  a.ns = L->n_ent;
  a.A = L->n_agents > 0 ? L->n_agents : L->n_ent;
  a.Q = a.A + 3;
  a.Lt = a.ns + a.A + 3;
  a.XS = L->E + 1;
  a.qpad = (a.Q + 15) / 16 * 16;
  if (a.A > 64 || a.Lt > 64 * TSLOT) return T2O_EUNSUPPORTED;
  for (a.waves = 4; a.waves >= 1; a.waves >>= 1) {
    lds = sizeof(float) * mix_lds_floats(a.Lt, a.XS, a.Q, L->E, a.ns, L->F, a.A, L->H, a.waves);
    if (lds <= 160 * 1024) return 0;
  }
  return T2O_EUNSUPPORTED;
}

int gen_mixer_unroll_fwd(const t2o_layout* L, const float* pack_on, const float* pack_tg, const float* states,
                         int64_t st_sb, int64_t st_st, const float* hid_on, const float* hid_tg, int64_t hid_sb,
                         int64_t hid_st, const float* hw0_on, const float* hw0_tg, int qmode_on, int qmode_tg,
                         const float* qv_on, const float* qv_tg, const float* q_on, const float* q_tg, int q_ts,
                         int n_actions, const int64_t* actions, int64_t act_sb, int64_t act_st,
                         const int32_t* avail, int64_t av_sb, int64_t av_st, float* y_on, float* hw_on,
                         float* qvo_on, float* xout_on, float* xmid_on, float* y_tg, float* hw_tg, float* qvo_tg,
                         float* xout_tg, float* xmid_tg, int B, int T_on, int T_tg, hipStream_t stream) {
  if (!gen_limits(*L)) return T2O_EUNSUPPORTED;
  GMixArgs a{};
  a.L = *L;
  a.g = gen_offsets(1, L->E, L->H, L->D, L->F, 1, L->FF);
  a.R = gen_rec(L->E, L->H, L->FF);
  size_t lds = 0;
  if (int rc = mixer_launch_dims(L, a, lds)) return rc;
  if ((qmode_on != 0 || (pack_tg && qmode_tg != 0)) && (n_actions < 1 || n_actions > 64)) return T2O_EUNSUPPORTED;
  a.states = states;
  a.st_sb = st_sb;
  a.st_st = st_st;
  a.hid_sb = hid_sb;
  a.hid_st = hid_st;
  a.qarg = q_on;
  a.q_ts = q_ts;
  a.n_actions = n_actions;
  a.actions = actions;
  a.act_sb = act_sb;
  a.act_st = act_st;
  a.avail = avail;
  a.av_sb = av_sb;
  a.av_st = av_st;
  a.B = B;
  a.net[0] = GMixNet{pack_on, hw0_on, hid_on, q_on, qv_on, qmode_on, T_on, y_on, hw_on, qvo_on, xout_on, xmid_on};
  int nnet = 1;
  if (pack_tg) {
    a.net[1] = GMixNet{pack_tg, hw0_tg, hid_tg, q_tg, qv_tg, qmode_tg, T_tg, y_tg, hw_tg, qvo_tg, xout_tg, xmid_tg};
    nnet = 2;
  }
  (void)hipFuncSetAttribute((const void*)gmixer_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(gmixer_fwd_kernel, dim3(B, nnet), dim3(64 * a.waves), lds, stream, a);
  return (int)hipGetLastError();
}

int gen_mixer_unroll_bwd(const t2o_layout* L, const float* pack, const float* states, int64_t st_sb, int64_t st_st,
                         const float* hid, int64_t hid_sb, int64_t hid_st, const float* hw0, const float* qv,
                         const float* hw, const float* xout, const float* xmid, const float* gy,
                         const float* ghw_ext, float* gqv, float* ghid, float* ghw0, float* gslabs, int max_slabs,
                         int* nslab, void* tape, int B, int T, hipStream_t stream) {
  if (!gen_limits(*L)) return T2O_EUNSUPPORTED;
  if (max_slabs < 1) return T2O_EINVAL;
  GMixArgs a{};
  a.L = *L;
  a.g = gen_offsets(1, L->E, L->H, L->D, L->F, 1, L->FF);
  a.R = gen_rec(L->E, L->H, L->FF);
  size_t lds = 0;
  if (int rc = mixer_launch_dims(L, a, lds)) return rc;
  a.states = states;
  a.st_sb = st_sb;
  a.st_st = st_st;
  a.hid_sb = hid_sb;
  a.hid_st = hid_st;
  a.net[0] = GMixNet{pack, hw0, hid, nullptr, qv, 0, T, nullptr, nullptr, nullptr, nullptr, nullptr};
  a.hw = hw;
  a.xout = xout;
  a.xmid = xmid;
  a.gy = gy;
  a.ghw_ext = ghw_ext;
  a.gqv = gqv;
  a.ghid = ghid;
  a.ghw0 = ghw0;
  a.slab = gslabs;
  a.tape = static_cast<float*>(tape);
  a.B = B;
  hipError_t e = hipMemsetAsync(gslabs, 0, sizeof(float) * (size_t)L->grad_total, stream);
  const int64_t tiles = (int64_t)B * T * (a.qpad / 16);
  if (e == hipSuccess) e = hipMemsetAsync(tape, 0, sizeof(float) * (size_t)gen_tape_floats(L, tiles), stream);
  if (e != hipSuccess) return (int)e;
  (void)hipFuncSetAttribute((const void*)gmixer_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(gmixer_bwd_kernel, dim3(B), dim3(64 * a.waves), lds, stream, a);
  *nslab = 1;
  return (int)hipGetLastError();
}

int gen_tape_contract(const t2o_layout* L, const void* tape, int64_t tiles, float* gslabs, int nslab,
                      hipStream_t stream) {
  if (nslab < 1) return T2O_EINVAL;
  const int E = L->E, H = L->H, FF = L->FF, HE = H * E;
  const GenOffsets g = gen_offsets(L->kind, E, H, L->D, L->F, L->kind == 0 ? L->NA : 1, FF);
  const GenRec R = gen_rec(E, H, FF);
  const int64_t nrec = tiles * 16;
  const float* base = static_cast<const float*>(tape);
  for (int d = 0; d < L->D; ++d) {
    const float* rec = base + (size_t)d * nrec * R.SIZE;
    const GemmTask tasks[6] = {
        {HE, E, 1, E, R.GQ, R.X, 0, 0, g.P.Wq[d], 0},                        // dWq = Σ gq ⊗ x
        {E, E, H, E, R.Q, R.GU, E, E, g.P.Wk[d], (int64_t)E * E},           // dWk_h = Σ q_h ⊗ gu_h
        {E, E, H, E, R.GV, R.Z, E, E, g.P.Wv[d], (int64_t)E * E},           // dWv_h = Σ gv_h ⊗ z_h
        {E, HE, 1, HE, R.GA, R.V, 0, 0, g.P.U[d], 0},                       // dU = Σ ga ⊗ v
        {FF, E, 1, E, R.GF1, R.Y, 0, 0, g.P.W1[d], 0},                      // dW1 = Σ gf1 ⊗ y
        {E, FF, 1, FF, R.GR2, R.FR, 0, 0, g.P.W2[d], 0},                    // dW2 = Σ gr2 ⊗ relu(f1)
    };
    for (const GemmTask& tk : tasks)
      if (int rc = launch_gemm(rec, nrec, R.SIZE, tk, gslabs, stream)) return rc;
  }
  return 0;
}

}  // namespace t2o
