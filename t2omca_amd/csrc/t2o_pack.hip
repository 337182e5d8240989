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
#include "t2o_layout.hpp"

using namespace t2o;

namespace {

enum SegKind : int {
  SEG_COPY = 0,     // dst[i] = src[i]
  SEG_PAD2D,        // dst[r][c] (R x C) = r<sr && c<sc ? src[r*sc + c] : 0
  SEG_TPAD2D,       // dst[r][c] (R x C) = c<sr && r<sc ? src[c*sc + r] : 0   (transpose of src[sr][sc])
  SEG_FOLD_M,       // dst[hE+i][k]   = s Σ_m Wk[hE+m][i] Wq[hE+m][k]
  SEG_FOLD_MT,      // dst[k][hE+i]   = same value
  SEG_FOLD_N,       // dst[o][hE+k]   = Σ_m U[o][hE+m] Wv[hE+m][k]
  SEG_FOLD_NT,      // dst[hE+k][o]
  SEG_ADD,          // dst[i] += src[i]
  SEG_ADD_PAD2D,    // dst[r][c] (r<R, c<C, ld C) += src[r*sc + c]   (src rows padded: ld sc)
  SEG_UNFOLD_WQ,    // dst(Wq)[hE+m][k] += s Σ_i Wk[hE+m][i] gM[hE+i][k]
  SEG_UNFOLD_WK,    // dst(Wk)[hE+m][i] += s Σ_k Wq[hE+m][k] gM[hE+i][k]
  SEG_UNFOLD_WV,    // dst(Wv)[hE+m][k] += Σ_o U[o][hE+m] gN[o][hE+k]
  SEG_UNFOLD_U,     // dst(U)[o][hE+m]  += Σ_k gN[o][hE+k] Wv[hE+m][k]
};

struct Seg {
  int kind;
  int R, C;        // destination rows / cols (n = R*C)
  int sr, sc;      // source dims (pad/transposes)
  int64_t dst, a, b;  // float offsets: dst in dst buffer; a/b in source buffers
};

// One launch per table keeps the kernel-argument block well under 4 KiB.
constexpr int MAX_SEGS = 24;
struct SegTable {
  int n;
  int E, H;
  float scale;
  Seg s[MAX_SEGS];
  int64_t start[MAX_SEGS + 1];
};

__global__ void seg_kernel(SegTable tab, const float* __restrict__ src, const float* __restrict__ src2,
                           float* __restrict__ dst) {
  const int64_t total = tab.start[tab.n];
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int k = 0;
    while (idx >= tab.start[k + 1]) ++k;
    const Seg sg = tab.s[k];
    const int64_t li = idx - tab.start[k];
    const int r = (int)(li / sg.C), cc = (int)(li % sg.C);
    const int E = tab.E;
    float v;
    switch (sg.kind) {
      case SEG_COPY: dst[sg.dst + li] = src[sg.a + li]; break;
      case SEG_PAD2D:
        dst[sg.dst + li] = (r < sg.sr && cc < sg.sc) ? src[sg.a + (int64_t)r * sg.sc + cc] : 0.f;
        break;
      case SEG_TPAD2D:
        dst[sg.dst + li] = (cc < sg.sr && r < sg.sc) ? src[sg.a + (int64_t)cc * sg.sc + r] : 0.f;
        break;
      case SEG_FOLD_M:
      case SEG_FOLD_MT: {
        // value M[row][col] with row = hE+i, col = k
        const int row = sg.kind == SEG_FOLD_M ? r : cc;
        const int col = sg.kind == SEG_FOLD_M ? cc : r;
        const int h = row / E, i = row % E;
        const float* Wk = src + sg.a + (int64_t)h * E * E;
        const float* Wq = src + sg.b + (int64_t)h * E * E;
        float acc = 0.f;
        for (int m = 0; m < E; ++m) acc = fmaf(Wk[m * E + i], Wq[m * E + col], acc);
        dst[sg.dst + li] = acc * tab.scale;
        break;
      }
      case SEG_FOLD_N:
      case SEG_FOLD_NT: {
        const int o = sg.kind == SEG_FOLD_N ? r : cc;
        const int hk = sg.kind == SEG_FOLD_N ? cc : r;
        const int h = hk / E, kk = hk % E;
        const int HE = tab.H * E;
        const float* U = src + sg.a;
        const float* Wv = src + sg.b + (int64_t)h * E * E;
        float acc = 0.f;
        for (int m = 0; m < E; ++m) acc = fmaf(U[(int64_t)o * HE + h * E + m], Wv[m * E + kk], acc);
        dst[sg.dst + li] = acc;
        break;
      }
      case SEG_ADD: dst[sg.dst + li] += src2[sg.a + li]; break;
      case SEG_ADD_PAD2D: dst[sg.dst + li] += src2[sg.a + (int64_t)r * sg.sc + cc]; break;
      case SEG_UNFOLD_WQ: {  // dst index (hE+m, k); src = params, src2 = gpack
        const int h = r / E, m = r % E;
        const float* Wk = src + sg.a + (int64_t)h * E * E;
        const float* gM = src2 + sg.b + (int64_t)h * E * E;
        float acc = 0.f;
        for (int i = 0; i < E; ++i) acc = fmaf(Wk[m * E + i], gM[i * E + cc], acc);
        dst[sg.dst + li] += acc * tab.scale;
        break;
      }
      case SEG_UNFOLD_WK: {  // dst index (hE+m, i)
        const int h = r / E, m = r % E;
        const float* Wq = src + sg.a + (int64_t)h * E * E;
        const float* gM = src2 + sg.b + (int64_t)h * E * E;
        float acc = 0.f;
        for (int kk = 0; kk < E; ++kk) acc = fmaf(Wq[m * E + kk], gM[cc * E + kk], acc);
        dst[sg.dst + li] += acc * tab.scale;
        break;
      }
      case SEG_UNFOLD_WV: {  // dst index (hE+m, k)
        const int h = r / E, m = r % E;
        const int HE = tab.H * E;
        const float* U = src + sg.a;
        const float* gN = src2 + sg.b;
        float acc = 0.f;
        for (int o = 0; o < E; ++o) acc = fmaf(U[(int64_t)o * HE + h * E + m], gN[(int64_t)o * HE + h * E + cc], acc);
        dst[sg.dst + li] += acc;
        break;
      }
      case SEG_UNFOLD_U: {  // dst index (o, hE+m)
        const int h = cc / E, m = cc % E;
        const int HE = tab.H * E;
        const float* Wv = src + sg.a + (int64_t)h * E * E;
        const float* gN = src2 + sg.b;
        float acc = 0.f;
        for (int kk = 0; kk < E; ++kk) acc = fmaf(gN[(int64_t)r * HE + h * E + kk], Wv[m * E + kk], acc);
        dst[sg.dst + li] += acc;
        break;
      }
      default: (void)v; break;
    }
  }
}

void add(SegTable& t, int kind, int R, int C, int64_t dst, int64_t a, int64_t b = 0, int sr = 0, int sc = 0) {
  Seg& s = t.s[t.n];
  s.kind = kind; s.R = R; s.C = C; s.sr = sr; s.sc = sc; s.dst = dst; s.a = a; s.b = b;
  t.start[t.n + 1] = t.start[t.n] + (int64_t)R * C;
  t.n++;
}

int launch(const SegTable& t, const float* src, const float* src2, float* dst, void* stream) {
  const int64_t total = t.start[t.n];
  if (total == 0) return 0;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(seg_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, t, src, src2, dst);
  return (int)hipGetLastError();
}

// bf16 image of the pack's matrices (round to nearest even), rows swizzled as
// bf_swz prescribes; blockIdx.y = matrix.  Vector slots of the image stay unused.
struct MatTable {
  int n;
  int64_t off[4 + 8 * T2O_MAX_DEPTH];
  int rows[4 + 8 * T2O_MAX_DEPTH], ld[4 + 8 * T2O_MAX_DEPTH];
};

__global__ void to_bf16_kernel(MatTable t, const float* __restrict__ src, __bf16* __restrict__ dst) {
  const int m = blockIdx.y;
  const int64_t off = t.off[m];
  const int ld = t.ld[m];
  const int64_t n = (int64_t)t.rows[m] * ld;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / ld), col = (int)(i % ld);
    dst[off + (int64_t)r * ld + (col ^ bf_swz(r, ld))] = (__bf16)src[off + i];
  }
}
}  // namespace

extern "C" int t2o_layout_init(t2o_layout* L, int kind, int E, int H, int D, int F, int NA, int FF, int n_ent,
                               int prec) {
  if (!L || (kind != 0 && kind != 1) || E <= 0 || E % 16 || H < 1 || D < 1 || D > T2O_MAX_DEPTH ||
      F < 1 || F > 16 || NA < 1 || NA > 16 || FF <= 0 || FF % 16 || n_ent < 1 || (prec != 0 && prec != 1))
    return T2O_EINVAL;
  t2o_layout z{};
  *L = z;
  L->kind = kind; L->E = E; L->H = H; L->D = D; L->F = F; L->NA = NA; L->FF = FF; L->n_ent = n_ent;
  L->prec = prec;
  int64_t o = 0;
  const int64_t HE = (int64_t)H * E;
  for (int d = 0; d < T2O_MAX_DEPTH; ++d)
    L->M[d] = L->MT[d] = L->N[d] = L->NT[d] = L->bu[d] = L->g1[d] = L->n1[d] = L->W1[d] = L->W1T[d] = L->c1[d] =
        L->W2[d] = L->W2T[d] = L->c2[d] = L->g2[d] = L->n2[d] = -1;
  // forward matrices, then forward vectors (one contiguous LDS copy; in bf16
  // mode the vectors stay fp32), then the backward's transposed copies.  Every
  // size is a multiple of 16 elements, so every section stays 64-B aligned.
  L->WeT = o; o += 16 * (int64_t)E;
  L->We = o; o += (int64_t)E * 16;
  L->Wo = o; o += 16 * (int64_t)E;
  for (int d = 0; d < D; ++d) {
    L->M[d] = o; o += HE * E;
    L->N[d] = o; o += E * HE;
    L->W1[d] = o; o += (int64_t)FF * E;
    L->W2[d] = o; o += (int64_t)E * FF;
  }
  L->vec_lo = o;
  L->be = o; o += E;
  L->bo = o; o += 16;
  for (int d = 0; d < D; ++d) {
    L->bu[d] = o; o += E;
    L->g1[d] = o; o += E;
    L->n1[d] = o; o += E;
    L->c1[d] = o; o += FF;
    L->c2[d] = o; o += E;
    L->g2[d] = o; o += E;
    L->n2[d] = o; o += E;
  }
  L->fwd_total = o;
  L->WoT = o; o += (int64_t)E * 16;
  for (int d = 0; d < D; ++d) {
    L->MT[d] = o; o += E * HE;
    L->NT[d] = o; o += HE * E;
    L->W1T[d] = o; o += (int64_t)E * FF;
    L->W2T[d] = o; o += (int64_t)FF * E;
  }
  L->total = o;
  L->pack_floats = prec ? o + ((o + 1) / 2 + 3) / 4 * 4 : o;
  t2o_layout G;
  grad_layout(*L, G);
  L->grad_total = G.grad_total;
  return 0;
}

extern "C" int t2o_layout_sizeof(void) { return (int)sizeof(t2o_layout); }

extern "C" int64_t t2o_param_count(int kind, int E, int H, int D, int F, int NA, int FF) {
  return param_offsets(kind, E, H, D, F, NA, FF).total;
}

extern "C" int t2o_pack_params(const t2o_layout* L, const float* params, float* pack, void* stream) {
  if (!L || !params || !pack) return T2O_EINVAL;
  const int E = L->E, H = L->H, D = L->D, F = L->F, FF = L->FF;
  const int HE = H * E;
  const ParamOffsets P = param_offsets(L->kind, E, H, D, F, L->NA, FF);
  SegTable t{};
  t.E = E; t.H = H; t.scale = 1.0f / sqrtf((float)E);
  add(t, SEG_TPAD2D, 16, E, L->WeT, P.We, 0, E, F);   // WeT[f][e] = We[e][f]
  add(t, SEG_PAD2D, E, 16, L->We, P.We, 0, E, F);
  add(t, SEG_COPY, 1, E, L->be, P.be);
  const int no = L->kind == 0 ? L->NA : 1;
  add(t, SEG_PAD2D, 16, E, L->Wo, P.Wo, 0, no, E);
  add(t, SEG_PAD2D, 1, 16, L->bo, P.bo, 0, 1, no);
  add(t, SEG_TPAD2D, E, 16, L->WoT, P.Wo, 0, no, E);
  for (int d = 0; d < D; ++d) {
    if (int rc = launch(t, params, nullptr, pack, stream)) return rc;
    t.n = 0;
    add(t, SEG_FOLD_M, HE, E, L->M[d], P.Wk[d], P.Wq[d]);
    add(t, SEG_FOLD_MT, E, HE, L->MT[d], P.Wk[d], P.Wq[d]);
    add(t, SEG_FOLD_N, E, HE, L->N[d], P.U[d], P.Wv[d]);
    add(t, SEG_FOLD_NT, HE, E, L->NT[d], P.U[d], P.Wv[d]);
    add(t, SEG_COPY, 1, E, L->bu[d], P.bu[d]);
    add(t, SEG_COPY, 1, E, L->g1[d], P.g1[d]);
    add(t, SEG_COPY, 1, E, L->n1[d], P.n1[d]);
    add(t, SEG_COPY, FF, E, L->W1[d], P.W1[d]);
    add(t, SEG_TPAD2D, E, FF, L->W1T[d], P.W1[d], 0, FF, E);
    add(t, SEG_COPY, 1, FF, L->c1[d], P.c1[d]);
    add(t, SEG_COPY, E, FF, L->W2[d], P.W2[d]);
    add(t, SEG_TPAD2D, FF, E, L->W2T[d], P.W2[d], 0, E, FF);
    add(t, SEG_COPY, 1, E, L->c2[d], P.c2[d]);
    add(t, SEG_COPY, 1, E, L->g2[d], P.g2[d]);
    add(t, SEG_COPY, 1, E, L->n2[d], P.n2[d]);
  }
  if (int rc = launch(t, params, nullptr, pack, stream)) return rc;
  if (L->prec == 1) {  // bf16 image of the matrices right after the fp32 pack
    MatTable m{};
    auto mat = [&](int64_t off, int rows, int ld) {
      m.off[m.n] = off;
      m.rows[m.n] = rows;
      m.ld[m.n] = ld;
      ++m.n;
    };
    mat(L->WeT, 16, E);
    mat(L->We, E, 16);
    mat(L->Wo, 16, E);
    mat(L->WoT, E, 16);
    for (int d = 0; d < D; ++d) {
      mat(L->M[d], HE, E);
      mat(L->MT[d], E, HE);
      mat(L->N[d], E, HE);
      mat(L->NT[d], HE, E);
      mat(L->W1[d], FF, E);
      mat(L->W1T[d], E, FF);
      mat(L->W2[d], E, FF);
      mat(L->W2T[d], FF, E);
    }
    hipLaunchKernelGGL(to_bf16_kernel, dim3(16, m.n), dim3(256), 0, (hipStream_t)stream, m, pack,
                       reinterpret_cast<__bf16*>(pack + L->total));
    return (int)hipGetLastError();
  }
  return 0;
}

extern "C" int t2o_unpack_grads(const t2o_layout* L, const float* params, const float* gpack, float* grad,
                                void* stream) {
  if (!L || !params || !gpack || !grad) return T2O_EINVAL;
  const int E = L->E, H = L->H, D = L->D, F = L->F, FF = L->FF;
  const int HE = H * E;
  const ParamOffsets P = param_offsets(L->kind, E, H, D, F, L->NA, FF);
  t2o_layout G;
  grad_layout(*L, G);
  SegTable t{};
  t.E = E; t.H = H; t.scale = 1.0f / sqrtf((float)E);
  // gWe[e][f] += gpack.We[e][f] (ld 16)
  add(t, SEG_ADD_PAD2D, E, F, P.We, G.We, 0, 0, 16);
  add(t, SEG_ADD, 1, E, P.be, G.be);
  const int no = L->kind == 0 ? L->NA : 1;
  add(t, SEG_ADD_PAD2D, no, E, P.Wo, G.Wo, 0, 0, E);
  add(t, SEG_ADD, 1, no, P.bo, G.bo);
  for (int d = 0; d < D; ++d) {
    if (int rc = launch(t, params, gpack, grad, stream)) return rc;
    t.n = 0;
    add(t, SEG_UNFOLD_WQ, HE, E, P.Wq[d], P.Wk[d], G.M[d]);
    add(t, SEG_UNFOLD_WK, HE, E, P.Wk[d], P.Wq[d], G.M[d]);
    add(t, SEG_UNFOLD_WV, HE, E, P.Wv[d], P.U[d], G.N[d]);
    add(t, SEG_UNFOLD_U, E, HE, P.U[d], P.Wv[d], G.N[d]);
    add(t, SEG_ADD, 1, E, P.bu[d], G.bu[d]);
    add(t, SEG_ADD, 1, E, P.g1[d], G.g1[d]);
    add(t, SEG_ADD, 1, E, P.n1[d], G.n1[d]);
    add(t, SEG_ADD, FF, E, P.W1[d], G.W1[d]);
    add(t, SEG_ADD, 1, FF, P.c1[d], G.c1[d]);
    add(t, SEG_ADD, E, FF, P.W2[d], G.W2[d]);
    add(t, SEG_ADD, 1, E, P.c2[d], G.c2[d]);
    add(t, SEG_ADD, 1, E, P.g2[d], G.g2[d]);
    add(t, SEG_ADD, 1, E, P.n2[d], G.n2[d]);
  }
  return launch(t, params, gpack, grad, stream);
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
