// t2o_pack.hip — parameter folding (params -> kernel pack), gradient unfolding
// (compact gradient block -> reference parameter grads) and slab reduction.
//
// Folding (per block d, head h; E = emb):
//   M_h = Wk_hᵀ · Wq_h / √E      scores_h(x, key) = (M_h x) · key
//   N_h = U_h · Wv_h             attended = Σ_h N_h z_h + b_U,  z_h = Σ p_h,j key_j
// This is transformer.py:52-84 re-associated: (Wq x / e^¼)·(Wk k / e^¼) and
// unify(concat_h Wv_h Σ p k) are the same bilinear forms.  The grads map back by
//   gWq_h = Wk_h gM_h /√E,  gWk_h = Wq_h gM_hᵀ /√E,  gWv_h = U_hᵀ gN_h,  gU_h = gN_h Wv_hᵀ.
#include <math.h>

#include "t2o_common.hpp"
#include "t2o_dispatch.hpp"
#include "t2o_layout.hpp"

using namespace t2o;

namespace {

// One launch per call: a table of tasks, each a range of workgroups.
//   elementwise tasks (copies, pads, transposes, grad adds): 1024 elements per
//     workgroup, optionally also writing the bf16 image of a matrix entry;
//   fold / unfold tasks: one workgroup per (block, head) E x E product, its
//     operands staged in LDS (each output is an E-long dot product from LDS).
enum TaskKind : int {
  T_COPY = 0,     // dst[i] = src[a + i]
  T_PAD2D,        // dst[r][c] (R x C) = r<sr && c<sc ? src[a + r*sc + c] : 0
  T_TPAD2D,       // dst[r][c] (R x C) = c<sr && r<sc ? src[a + c*sc + r] : 0   (transpose of src[sr][sc])
  T_ADD,          // dst[i] += src2[a + i]
  T_ADD_PAD2D,    // dst[r][c] (R x C, ld C) += src2[a + r*sc + c]
  T_FOLD_M,       // head h: M[hE+i][k] = MT[k][hE+i] = s Σ_m Wk[hE+m][i] Wq[hE+m][k]
  T_FOLD_N,       // head h: N[o][hE+k] = NT[hE+k][o] = Σ_m U[o][hE+m] Wv[hE+m][k]
  T_UNFOLD_QK,    // head h: gWq[hE+m][k] += s Σ_i Wk[hE+m][i] gM[hE+i][k]; gWk[hE+m][i] += s Σ_k Wq[hE+m][k] gM[hE+i][k]
  T_UNFOLD_VU,    // head h: gWv[hE+m][k] += Σ_o U[o][hE+m] gN[o][hE+k];  gU[o][hE+m] += Σ_k gN[o][hE+k] Wv[hE+m][k]
  T_UNFOLD_LN1,   // block: the LN1 / W1 grads from the contraction's P, Q (TapeRec, t2o_common.hpp)
};

struct Task {
  int kind;
  int R, C;          // elementwise: destination rows / cols
  int sr, sc;        // source dims (pads / transposes)
  int h, bf;         // head (fold tasks); bf: also write the bf16 image (ld = C)
  int64_t dst, dst2; // destination offsets (fold: M and MT, or N and NT; unfold: the two grads)
  int64_t a, b, c;   // source offsets
};

constexpr int MAX_TASKS = 40;
constexpr int EW_PER_BLOCK = 1024;
struct TaskTable {
  int n, E, H;
  float scale;
  Task t[MAX_TASKS];
  int blk[MAX_TASKS + 1];  // first workgroup of each task
};

T2O_DEV void put(float* dst, __bf16* dstb, int64_t off, int r, int col, int ld, float v, bool bf) {
  dst[off + (int64_t)r * ld + col] = v;
  if (bf) dstb[off + (int64_t)r * ld + (col ^ bf_swz(r, ld))] = (__bf16)v;
}

// an E x E operand (row stride ld) into LDS
// E x E block of g (leading dim ld) into LDS rows of stride E + 1: the
// products below read both rows and columns, and the odd stride keeps a
// wave's column reads on distinct banks
T2O_DEV void stage(float* s, const float* g, int E, int ld) {
  // (unrolled: a thread's loads issue together instead of one round trip each)
#pragma unroll 4
  for (int i = threadIdx.x; i < E * E; i += blockDim.x) s[(i / E) * (E + 1) + i % E] = g[(int64_t)(i / E) * ld + i % E];
}

__global__ __launch_bounds__(256) void pack_kernel(TaskTable tab, const float* __restrict__ src,
                                                   const float* __restrict__ src2, float* __restrict__ dst,
                                                   __bf16* __restrict__ dstb) {
  extern __shared__ float sm[];
  T2O_LDS_POISON(sm);
  int k = 0;
  while ((int)blockIdx.x >= tab.blk[k + 1]) ++k;
  const Task tk = tab.t[k];
  const int lb = (int)blockIdx.x - tab.blk[k];
  const int E = tab.E, HE = tab.H * E, h = tk.h;
  const int LS = E + 1, SQ = E * LS;  // staged matrix row stride / size (stage())
  const bool bf = tk.bf != 0;
  switch (tk.kind) {
    case T_COPY:
    case T_PAD2D:
    case T_TPAD2D:
    case T_ADD:
    case T_ADD_PAD2D: {
      const int64_t n = (int64_t)tk.R * tk.C;
      for (int64_t li = (int64_t)lb * EW_PER_BLOCK + threadIdx.x; li < n && li < (int64_t)(lb + 1) * EW_PER_BLOCK;
           li += blockDim.x) {
        const int r = (int)(li / tk.C), cc = (int)(li % tk.C);
        float v;
        if (tk.kind == T_COPY) v = src[tk.a + li];
        else if (tk.kind == T_PAD2D) v = (r < tk.sr && cc < tk.sc) ? src[tk.a + (int64_t)r * tk.sc + cc] : 0.f;
        else if (tk.kind == T_TPAD2D) v = (cc < tk.sr && r < tk.sc) ? src[tk.a + (int64_t)cc * tk.sc + r] : 0.f;
        else if (tk.kind == T_ADD) v = dst[tk.dst + li] + src2[tk.a + li];
        else v = dst[tk.dst + li] + src2[tk.a + (int64_t)r * tk.sc + cc];
        put(dst, dstb, tk.dst, r, cc, tk.C, v, bf);
      }
      break;
    }
    case T_FOLD_M: {  // a = Wk, b = Wq (params, [HE][E] row-major)
      float* wk = sm;
      float* wq = sm + SQ;
      stage(wk, src + tk.a + (int64_t)h * E * E, E, E);
      stage(wq, src + tk.b + (int64_t)h * E * E, E, E);
      __syncthreads();
      for (int o = threadIdx.x; o < E * E; o += blockDim.x) {
        const int i = o / E, kk = o % E;
        float acc = 0.f;
        for (int m = 0; m < E; ++m) acc = fmaf(wk[m * LS + i], wq[m * LS + kk], acc);
        acc *= tab.scale;
        put(dst, dstb, tk.dst, h * E + i, kk, E, acc, bf);   // M  [HE][E]
        put(dst, dstb, tk.dst2, kk, h * E + i, HE, acc, bf); // MT [E][HE]
      }
      break;
    }
    case T_FOLD_N: {  // a = U ([E][HE]), b = Wv ([HE][E])
      float* u = sm;
      float* wv = sm + SQ;
      stage(u, src + tk.a + (int64_t)h * E, E, HE);
      stage(wv, src + tk.b + (int64_t)h * E * E, E, E);
      __syncthreads();
      for (int o = threadIdx.x; o < E * E; o += blockDim.x) {
        const int oo = o / E, kk = o % E;
        float acc = 0.f;
        for (int m = 0; m < E; ++m) acc = fmaf(u[oo * LS + m], wv[m * LS + kk], acc);
        put(dst, dstb, tk.dst, oo, h * E + kk, HE, acc, bf);   // N  [E][HE]
        put(dst, dstb, tk.dst2, h * E + kk, oo, E, acc, bf);   // NT [HE][E]
      }
      break;
    }
    case T_UNFOLD_QK: {  // a = Wq, b = Wk (params), c = gM (gpack [HE][E]); dst = gWq, dst2 = gWk
      float* wq = sm;
      float* wk = sm + SQ;
      float* gm = sm + 2 * SQ;
      stage(wq, src + tk.a + (int64_t)h * E * E, E, E);
      stage(wk, src + tk.b + (int64_t)h * E * E, E, E);
      stage(gm, src2 + tk.c + (int64_t)h * E * E, E, E);
      __syncthreads();
      for (int o = threadIdx.x; o < E * E; o += blockDim.x) {
        const int m = o / E, kk = o % E;
        float aq = 0.f, ak = 0.f;
        for (int i = 0; i < E; ++i) {
          aq = fmaf(wk[m * LS + i], gm[i * LS + kk], aq);  // gWq[m][kk]
          ak = fmaf(wq[m * LS + i], gm[kk * LS + i], ak);  // gWk[m][kk] (kk plays i)
        }
        dst[tk.dst + (int64_t)(h * E + m) * E + kk] += aq * tab.scale;
        dst[tk.dst2 + (int64_t)(h * E + m) * E + kk] += ak * tab.scale;
      }
      break;
    }
    case T_UNFOLD_VU: {  // a = U, b = Wv (params), c = gN (gpack [E][HE]); dst = gWv, dst2 = gU
      float* u = sm;
      float* wv = sm + SQ;
      float* gn = sm + 2 * SQ;
      stage(u, src + tk.a + (int64_t)h * E, E, HE);
      stage(wv, src + tk.b + (int64_t)h * E * E, E, E);
      stage(gn, src2 + tk.c + (int64_t)h * E, E, HE);
      __syncthreads();
      for (int o = threadIdx.x; o < E * E; o += blockDim.x) {
        const int m = o / E, kk = o % E;
        float av = 0.f, au = 0.f;
        for (int j = 0; j < E; ++j) {
          av = fmaf(u[j * LS + m], gn[j * LS + kk], av);   // gWv[m][kk] = Σ_o U[o][m] gN[o][kk]
          au = fmaf(gn[m * LS + j], wv[kk * LS + j], au);  // gU[m][kk] = Σ_k gN[m][k] Wv[kk][k]  (m = o, kk = m')
        }
        dst[tk.dst + (int64_t)(h * E + m) * E + kk] += av;
        dst[tk.dst2 + (int64_t)m * HE + h * E + kk] += au;
      }
      break;
    }
    case T_UNFOLD_LN1: {
      // a / b / c = W1 [R=FF][C=E], g1, n1 (params; the grads sit at the same offsets);
      // gpack: dst = P [FF][E], dst2 = Q [E], sr = d c1 [FF], sc = d c2 [E].
      //   dW1 = P ⊙ g1 + d c1 ⊗ n1,  d g1 = Q + Σ_J W1[J] ⊙ P[J],  d n1 = d c2 + W1ᵀ d c1
      // workgroup 0: the two column sums; workgroups 1..: dW1, EW_PER_BLOCK entries each
      const int FFn = tk.R, En = tk.C;
      const float* W1 = src + tk.a;
      const float* g1 = src + tk.b;
      const float* n1 = src + tk.c;
      const float* Pm = src2 + tk.dst;
      const float* dc1 = src2 + tk.sr;
      if (lb > 0) {
        const int64_t n = (int64_t)FFn * En, i0 = (int64_t)(lb - 1) * EW_PER_BLOCK;
#pragma unroll 4
        for (int64_t i = i0 + threadIdx.x; i < n && i < i0 + EW_PER_BLOCK; i += blockDim.x) {
          const int J = (int)(i / En), e = (int)(i % En);
          dst[tk.a + i] += Pm[i] * g1[e] + dc1[J] * n1[e];
        }
        break;
      }
      // column sums over J: thread (q, e) takes J = q, q + NQ, ... ; partials in LDS
      const int NQ = (int)blockDim.x / En;
      float* part = sm;  // [2][NQ][E]
      if ((int)threadIdx.x < NQ * En) {
        const int e = threadIdx.x % En, q = threadIdx.x / En;
        float sg = 0.f, sn = 0.f;
#pragma unroll 4
        for (int J = q; J < FFn; J += NQ) {
          const float w = W1[(int64_t)J * En + e];
          sg = fmaf(w, Pm[(int64_t)J * En + e], sg);
          sn = fmaf(w, dc1[J], sn);
        }
        part[q * En + e] = sg;
        part[(NQ + q) * En + e] = sn;
      }
      __syncthreads();
      if ((int)threadIdx.x < En) {
        const int e = threadIdx.x;
        float sg = 0.f, sn = 0.f;
        for (int q = 0; q < NQ; ++q) {
          sg += part[q * En + e];
          sn += part[(NQ + q) * En + e];
        }
        dst[tk.b + e] += src2[tk.dst2 + e] + sg;
        dst[tk.c + e] += src2[tk.sc + e] + sn;
      }
      break;
    }
    default: break;
  }
}

// Collects tasks and launches them (several launches only when a table fills:
// the kernel-argument block stays under 4 KiB).
struct Builder {
  TaskTable tab{};
  int nb = 0, rc = 0;
  const float* src;
  const float* src2;
  float* dst;
  __bf16* dstb;
  void* stream;
  Builder(int E, int H, const float* s, const float* s2, float* d, __bf16* db, void* st)
      : src(s), src2(s2), dst(d), dstb(db), stream(st) {
    tab.E = E;
    tab.H = H;
    tab.scale = 1.0f / sqrtf((float)E);
  }
  Task& next(int blocks) {
    if (tab.n == MAX_TASKS) flush();
    Task& t = tab.t[tab.n];
    t = Task{};
    tab.blk[tab.n] = nb;
    nb += blocks;
    tab.blk[++tab.n] = nb;
    return t;
  }
  void ew(int kind, int R, int C, int64_t dst_off, int64_t a, int sr = 0, int sc = 0, int bf = 0) {
    Task& t = next((int)(((int64_t)R * C + EW_PER_BLOCK - 1) / EW_PER_BLOCK));
    t.kind = kind; t.R = R; t.C = C; t.sr = sr; t.sc = sc; t.bf = bf; t.dst = dst_off; t.a = a;
  }
  void head(int kind, int h, int64_t dst_off, int64_t dst2_off, int64_t a, int64_t b, int64_t c = 0, int bf = 0) {
    Task& t = next(1);
    t.kind = kind; t.h = h; t.bf = bf; t.dst = dst_off; t.dst2 = dst2_off; t.a = a; t.b = b; t.c = c;
  }
  // T_UNFOLD_LN1: per block, one workgroup for the column sums plus the dW1 workgroups
  void ln1(int64_t w1, int64_t g1, int64_t n1, int64_t gP, int64_t gQ, int64_t gc1, int64_t gc2, int FF, int E) {
    Task& t = next(1 + (int)(((int64_t)FF * E + EW_PER_BLOCK - 1) / EW_PER_BLOCK));
    t.kind = T_UNFOLD_LN1; t.R = FF; t.C = E; t.a = w1; t.b = g1; t.c = n1; t.dst = gP; t.dst2 = gQ;
    t.sr = (int)gc1; t.sc = (int)gc2;
  }
  void flush() {
    if (nb > 0 && rc == 0) {
      const size_t lds = sizeof(float) * 3 * (size_t)tab.E * (tab.E + 1);
      hipLaunchKernelGGL(pack_kernel, dim3(nb), dim3(256), lds, (hipStream_t)stream, tab, src, src2, dst, dstb);
      rc = (int)hipGetLastError();
    }
    tab.n = 0;
    nb = 0;
  }
  int finish() {
    flush();
    return rc;
  }
};
}  // namespace

extern "C" int t2o_layout_instance(const t2o_layout* L) {
  if (!L) return T2O_EINVAL;
  if (L->generic) return T2O_INSTANCE_GENERIC;
  const bool abs_head = L->kind == 0 || L->pos_func == T2O_POS_ABS;  // (exact mixer instances: abs head,
  // and at 8 AGVs every head: t2o_dispatch.hpp T2O_DISPATCH_MIXER)
  const bool exact_8 = L->kind == 1 && L->n_ent == 8 && t2o_default_net(L->E, L->H, L->D, L->FF);
  return (abs_head || exact_8) && t2o_exact_shape(L->E, L->H, L->D, L->n_ent, L->FF) ? T2O_INSTANCE_EXACT
                                                                                      : T2O_INSTANCE_RUNTIME;
}

extern "C" int t2o_layout_init(t2o_layout* L, int kind, int E, int H, int D, int F, int NA, int FF, int n_ent,
                               int prec) {
  return t2o_layout_init_ex(L, kind, E, H, D, F, NA, FF, n_ent, prec, 0, T2O_POS_ABS, 1.0f, 0);
}

extern "C" int t2o_layout_init_ex(t2o_layout* L, int kind, int E, int H, int D, int F, int NA, int FF, int n_ent,
                                  int prec, int n_agents, int pos_func, float pos_beta, int flags) {
  if (!L || (kind != 0 && kind != 1) || E <= 0 || H < 1 || D < 1 || D > T2O_MAX_DEPTH || F < 1 || F > 16 ||
      NA < 1 || NA > 16 || FF <= 0 || n_ent < 1 || (prec != 0 && prec != 1) || pos_func < 0 || pos_func > 3 ||
      !(pos_beta > 0.f))
    return T2O_EINVAL;
  if (n_agents <= 0) n_agents = n_ent;
  if (kind == 0 && n_agents != n_ent) return T2O_EINVAL;  // the agent's rows are its own sequences
  t2o_layout z{};
  *L = z;
  L->kind = kind; L->E = E; L->H = H; L->D = D; L->F = F; L->NA = NA; L->FF = FF; L->n_ent = n_ent;
  L->prec = prec;
  L->n_agents = n_agents;
  L->pos_func = pos_func;
  L->pos_beta = pos_beta;
  for (int d = 0; d < T2O_MAX_DEPTH; ++d)
    L->M[d] = L->MT[d] = L->N[d] = L->NT[d] = L->bu[d] = L->g1[d] = L->n1[d] = L->W1[d] = L->W1T[d] = L->c1[d] =
        L->W2[d] = L->W2T[d] = L->c2[d] = L->g2[d] = L->n2[d] = -1;
  // the exact mixer instances compute pos_func abs only (the reference default);
  // the runtime-entity instances take it as a parameter, so the default network
  // runs every qmix_pos_func on MFMA kernels (t2o_dispatch.hpp), other networks
  // with a non-abs head run the generic kernels
  if ((flags & T2O_LAYOUT_FORCE_GENERIC) || n_agents != n_ent || !t2o_tuned_shape(E, H, D, n_ent, FF) ||
      (kind == 1 && pos_func != T2O_POS_ABS && !t2o_default_net(E, H, D, FF))) {
    // runtime-shaped kernels (t2o_generic.hip): pack = reference-order params +
    // transposed copies; compact grads = reference order
    const bool ok = E <= 64 && H <= 8 && H * E <= 512 && FF <= 512 &&
                    (kind == 0 ? n_ent <= 64 : (n_agents <= 64 && n_ent + n_agents + 3 <= 192));
    if (!ok) return T2O_EUNSUPPORTED;
    L->generic = 1;
    L->WeT = L->We = L->be = L->Wo = L->bo = L->WoT = -1;
    const GenOffsets g = gen_offsets(kind, E, H, D, F, kind == 0 ? NA : 1, FF);
    L->vec_lo = 0;
    L->fwd_total = L->total = L->pack_floats = g.total;
    L->grad_total = g.P.total;
    return 0;
  }
  tuned_pack_offsets(*L, E, H, D, FF, prec);  // (t2o_layout.hpp: also the kernels' compile-time copy)
  return 0;
}

extern "C" int t2o_layout_sizeof(void) { return (int)sizeof(t2o_layout); }

extern "C" int t2o_args_sizeof(int which) {
  switch (which) {
    case T2O_ARGS_AGENT_FWD: return (int)sizeof(t2o_agent_fwd_args);
    case T2O_ARGS_AGENT_BWD: return (int)sizeof(t2o_agent_bwd_args);
    case T2O_ARGS_MIXER_FWD: return (int)sizeof(t2o_mixer_fwd_args);
    case T2O_ARGS_MIXER_BWD: return (int)sizeof(t2o_mixer_bwd_args);
    case T2O_ARGS_TAPE: return (int)sizeof(t2o_tape_args);
    case T2O_ARGS_TD: return (int)sizeof(t2o_td_args);
    default: return -1;
  }
}

extern "C" int t2o_abi_version(void) { return T2O_ABI_VERSION; }

extern "C" int64_t t2o_param_count(int kind, int E, int H, int D, int F, int NA, int FF) {
  return param_offsets(kind, E, H, D, F, NA, FF).total;
}

extern "C" int t2o_pack_params(const t2o_layout* L, const float* params, float* pack, void* stream) {
  if (!L || !params || !pack) return T2O_EINVAL;
  const int E = L->E, H = L->H, D = L->D, F = L->F, FF = L->FF;
  if (L->generic) {  // reference-order params, then the transposed copies (GenOffsets)
    const int no = L->kind == 0 ? L->NA : 1, HE = H * E;
    const GenOffsets g = gen_offsets(L->kind, E, H, D, F, no, FF);
    Builder b(E, H, params, nullptr, pack, nullptr, stream);
    b.ew(T_COPY, 1, (int)g.P.total, 0, 0);
    for (int d = 0; d < D; ++d) {
      b.ew(T_TPAD2D, E, HE, g.WqT[d], g.P.Wq[d], HE, E);
      b.ew(T_TPAD2D, E, HE, g.WkT[d], g.P.Wk[d], HE, E);
      b.ew(T_TPAD2D, E, HE, g.WvT[d], g.P.Wv[d], HE, E);
      b.ew(T_TPAD2D, HE, E, g.UT[d], g.P.U[d], E, HE);
      b.ew(T_TPAD2D, E, FF, g.W1T[d], g.P.W1[d], FF, E);
      b.ew(T_TPAD2D, FF, E, g.W2T[d], g.P.W2[d], E, FF);
    }
    b.ew(T_TPAD2D, F, E, g.WeT, g.P.We, E, F);
    b.ew(T_TPAD2D, E, no, g.WoT, g.P.Wo, no, E);
    return b.finish();
  }
  if (E > 64) return T2O_EUNSUPPORTED;
  const ParamOffsets P = param_offsets(L->kind, E, H, D, F, L->NA, FF);
  // bf16 mode: every matrix also goes to the swizzled bf16 image after the fp32 pack
  const int bf = L->prec == 1;
  __bf16* img = bf ? reinterpret_cast<__bf16*>(pack + L->total) : nullptr;
  Builder b(E, H, params, nullptr, pack, img, stream);
  b.ew(T_TPAD2D, 16, E, L->WeT, P.We, E, F, bf);   // WeT[f][e] = We[e][f]
  b.ew(T_PAD2D, E, 16, L->We, P.We, E, F, bf);
  b.ew(T_COPY, 1, E, L->be, P.be);
  const int no = L->kind == 0 ? L->NA : 1;
  b.ew(T_PAD2D, 16, E, L->Wo, P.Wo, no, E, bf);
  b.ew(T_PAD2D, 1, 16, L->bo, P.bo, 1, no);
  b.ew(T_TPAD2D, E, 16, L->WoT, P.Wo, no, E, bf);
  for (int d = 0; d < D; ++d) {
    for (int h = 0; h < H; ++h) {
      b.head(T_FOLD_M, h, L->M[d], L->MT[d], P.Wk[d], P.Wq[d], 0, bf);
      b.head(T_FOLD_N, h, L->N[d], L->NT[d], P.U[d], P.Wv[d], 0, bf);
    }
    b.ew(T_COPY, 1, E, L->bu[d], P.bu[d]);
    b.ew(T_COPY, 1, E, L->g1[d], P.g1[d]);
    b.ew(T_COPY, 1, E, L->n1[d], P.n1[d]);
    b.ew(T_COPY, FF, E, L->W1[d], P.W1[d], 0, 0, bf);
    b.ew(T_TPAD2D, E, FF, L->W1T[d], P.W1[d], FF, E, bf);
    b.ew(T_COPY, 1, FF, L->c1[d], P.c1[d]);
    b.ew(T_COPY, E, FF, L->W2[d], P.W2[d], 0, 0, bf);
    b.ew(T_TPAD2D, FF, E, L->W2T[d], P.W2[d], E, FF, bf);
    b.ew(T_COPY, 1, E, L->c2[d], P.c2[d]);
    b.ew(T_COPY, 1, E, L->g2[d], P.g2[d]);
    b.ew(T_COPY, 1, E, L->n2[d], P.n2[d]);
  }
  return b.finish();
}

extern "C" int t2o_unpack_grads(const t2o_layout* L, const float* params, const float* gpack, float* grad,
                                void* stream) {
  if (!L || !params || !gpack || !grad) return T2O_EINVAL;
  const int E = L->E, H = L->H, D = L->D, F = L->F, FF = L->FF;
  if (L->generic) {  // the generic backward's grads are already in reference order
    Builder b(E, H, params, gpack, grad, nullptr, stream);
    b.ew(T_ADD, 1, (int)L->grad_total, 0, 0);
    return b.finish();
  }
  if (E > 64) return T2O_EUNSUPPORTED;
  const ParamOffsets P = param_offsets(L->kind, E, H, D, F, L->NA, FF);
  t2o_layout G;
  grad_layout(*L, G);
  Builder b(E, H, params, gpack, grad, nullptr, stream);
  // gWe[e][f] += gpack.We[e][f] (ld 16)
  b.ew(T_ADD_PAD2D, E, F, P.We, G.We, 0, 16);
  b.ew(T_ADD, 1, E, P.be, G.be);
  const int no = L->kind == 0 ? L->NA : 1;
  b.ew(T_ADD_PAD2D, no, E, P.Wo, G.Wo, 0, E);
  b.ew(T_ADD, 1, no, P.bo, G.bo);
  for (int d = 0; d < D; ++d) {
    for (int h = 0; h < H; ++h) {
      b.head(T_UNFOLD_QK, h, P.Wq[d], P.Wk[d], P.Wq[d], P.Wk[d], G.M[d]);
      b.head(T_UNFOLD_VU, h, P.Wv[d], P.U[d], P.U[d], P.Wv[d], G.N[d]);
    }
    b.ew(T_ADD, 1, E, P.bu[d], G.bu[d]);
    b.ln1(P.W1[d], P.g1[d], P.n1[d], G.W1[d], G.g1[d], G.c1[d], G.c2[d], FF, E);
    b.ew(T_ADD, 1, FF, P.c1[d], G.c1[d]);
    b.ew(T_ADD, E, FF, P.W2[d], G.W2[d]);
    b.ew(T_ADD, 1, E, P.c2[d], G.c2[d]);
    b.ew(T_ADD, 1, E, P.g2[d], G.g2[d]);
    b.ew(T_ADD, 1, E, P.n2[d], G.n2[d]);
  }
  return b.finish();
}

namespace {
// out[i] = Σ_k slabs[k][i].  A block covers 64 columns as 16 column quads x 16
// slab lanes: each thread sums every 16th slab of its quad with 16-byte loads
// (independent, so many are in flight), then the 16 partials of a quad are
// combined through LDS in a fixed order (deterministic).
constexpr int RS_QUADS = 16, RS_LANES = 16;
__global__ __launch_bounds__(256) void reduce_slabs_kernel(const float* __restrict__ slabs, int nslab, int64_t n,
                                                           float* __restrict__ out) {
  __shared__ f4 part[RS_LANES][RS_QUADS];
  const int qd = threadIdx.x % RS_QUADS, ln = threadIdx.x / RS_QUADS;
  const int64_t col = ((int64_t)blockIdx.x * RS_QUADS + qd) * 4;
  f4 s = f4{0.f, 0.f, 0.f, 0.f};
  if (col + 3 < n && (n & 3) == 0) {
#pragma unroll 4
    for (int k = ln; k < nslab; k += RS_LANES) s += *reinterpret_cast<const f4*>(slabs + (int64_t)k * n + col);
  } else {
    for (int k = ln; k < nslab; k += RS_LANES)
      for (int r = 0; r < 4; ++r)
        if (col + r < n) s[r] += slabs[(int64_t)k * n + col + r];
  }
  part[ln][qd] = s;
  __syncthreads();
  if (ln == 0) {
    f4 t = part[0][qd];
    for (int l = 1; l < RS_LANES; ++l) t += part[l][qd];
    for (int r = 0; r < 4; ++r)
      if (col + r < n) out[col + r] = t[r];
  }
}
}  // namespace

extern "C" int t2o_reduce_slabs(const float* slabs, int nslab, int64_t n, float* out, void* stream) {
  if (!slabs || !out || nslab < 1 || n < 1) return T2O_EINVAL;
  const int64_t blocks = (n + 4 * RS_QUADS - 1) / (4 * RS_QUADS);
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, slabs, nslab, n, out);
  return (int)hipGetLastError();
}

// diagnostic: the bf16 image swizzle (tests check the image and its bank model)
extern "C" int t2o_bf_swz(int row, int ld) { return t2o::bf_swz(row, ld); }
