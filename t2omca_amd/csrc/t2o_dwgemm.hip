// t2o_dwgemm.hip — contraction of the weight-gradient tape (TapeRec, t2o_common.hpp).
//
// dM = Σ_n gu_n x_nᵀ,  dN = Σ_n gres_n z_nᵀ,  dW1 = Σ_n gf1_n y_nᵀ,  dW2 = Σ_n gr2_n f1r_nᵀ
// over every record (row x step of the agent, query row x step of the mixer)
// of every block.  This is a tall-skinny GEMM with K = records: split-K over
// workgroups (workgroup k contracts one contiguous range of 16-record tiles and
// writes the four matrices of every block into gradient slab k, whose
// small-gradient part the backward kernel has already filled), and inside a
// workgroup one wave per (block, matrix pair) keeps its 28 output tiles in MFMA
// accumulators for the whole range.  The tape is feature-major inside a tile
// (TapeRec), so one lane's K-slice is contiguous:
//   bf16: lane (g, c) loads 8 records (tile t0 + g/2, records 8(g&1)..+7) of
//         feature 16o+c as one 16-B load -> v_mfma_f32_16x16x32_bf16, 32 records
//   fp32: lane (g, c) loads records 4g..4g+3 of one tile (16 B) and feeds them
//         to four v_mfma_f32_16x16x4_f32, 16 records
// Bound: HBM (each record is read once: 1152 B (bf16) / 2304 B (fp32) per block).
// Called by the host right after t2o_agent_unroll_bwd / t2o_mixer_unroll_bwd
// with the same slabs: it fills their M/N/W1/W2 regions.
#include "t2o_common.hpp"
#include "t2o_dispatch.hpp"
#include "t2o_layout.hpp"

namespace t2o {

struct DwGemmArgs {
  const void* tape;    // [D][ntiles][SIZE][16]
  int64_t ntiles;      // 16-record tiles per block
  int64_t chunk;       // tiles per workgroup (multiple of 2)
  float* slabs;        // [nslab][slab_stride], compact gradient layout G
  int64_t slab_stride;
  t2o_layout G;
  int D;
};

template <int OT, int IT>
T2O_DEV void dw_tiles_store(float* __restrict__ W, int ldw, const f4 (&acc)[OT][IT]) {
  const int c = lane_c(), g = lane_g();
#pragma unroll
  for (int o = 0; o < OT; ++o)
#pragma unroll
    for (int i = 0; i < IT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) W[(16 * o + 4 * g + r) * ldw + 16 * i + c] = acc[o][i][r];
}

typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

// one operand pair over one K-step: acc[o][i] += Σ_k dY[k][16o+c] X[k][16i+c]
// fp32: `p` = this lane's tile base + its 4-record offset; K-step = 16 records
template <int OT, int IT>
T2O_DEV void dw_pair(f4 (&acc)[OT][IT], const float* __restrict__ p, bool ok, int offA, int offB) {
  const int c = lane_c();
  f4 a[OT], b[IT];
#pragma unroll
  for (int o = 0; o < OT; ++o) a[o] = ok ? ld4(p + (offA + 16 * o + c) * 16) : zero4();
#pragma unroll
  for (int i = 0; i < IT; ++i) b[i] = ok ? ld4(p + (offB + 16 * i + c) * 16) : zero4();
#pragma unroll
  for (int o = 0; o < OT; ++o)
#pragma unroll
    for (int i = 0; i < IT; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[o][i] = mfma4(a[o][s], b[i][s], acc[o][i]);
}
// bf16: K-step = 32 records (two tiles)
template <int OT, int IT>
T2O_DEV void dw_pair(f4 (&acc)[OT][IT], const __bf16* __restrict__ p, bool ok, int offA, int offB) {
  const int c = lane_c();
  const bf8v z{};
  bf8v a[OT], b[IT];
#pragma unroll
  for (int o = 0; o < OT; ++o) a[o] = ok ? *reinterpret_cast<const bf8v*>(p + (offA + 16 * o + c) * 16) : z;
#pragma unroll
  for (int i = 0; i < IT; ++i) b[i] = ok ? *reinterpret_cast<const bf8v*>(p + (offB + 16 * i + c) * 16) : z;
#pragma unroll
  for (int o = 0; o < OT; ++o)
#pragma unroll
    for (int i = 0; i < IT; ++i) acc[o][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[o], b[i], acc[o][i], 0, 0, 0);
}

// KIND (0 agent, 1 mixer) only separates the two instances in profiles.
template <int E, int H, int FF, int KIND, typename TT>
__global__ __launch_bounds__(64 * 2 * T2O_MAX_DEPTH) void dw_gemm_kernel(DwGemmArgs a) {
  using R = TapeRec<E, H, FF>;
  constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
  constexpr bool BF = sizeof(TT) == 2;
  const int w = wave_id();
  const int d = w >> 1;
  if (d >= a.D) return;
  const int g = lane_g();
  const int64_t t0 = (int64_t)blockIdx.x * a.chunk;
  const int64_t t1 = t0 + a.chunk < a.ntiles ? t0 + a.chunk : a.ntiles;
  const TT* __restrict__ base = static_cast<const TT*>(a.tape) + (size_t)d * a.ntiles * R::SIZE * 16;
  float* slab = a.slabs + (size_t)blockIdx.x * a.slab_stride;
  // this lane's K-slice inside a step: bf16 -> tile t + g/2, records 8(g&1)..;
  // fp32 -> tile t, records 4g..4g+3
  auto lane_ptr = [&](int64_t t, bool& ok) {
    const int64_t tt = BF ? t + (g >> 1) : t;
    ok = tt < t1;
    return base + (size_t)(ok ? tt : t0) * R::SIZE * 16 + (BF ? 8 * (g & 1) : 4 * g);
  };
  constexpr int STEP = BF ? 2 : 1;  // tiles per K-step
  if ((w & 1) == 0) {  // M (gu ⊗ x) and W1 (gf1 ⊗ y)
    f4 accM[HET][ET], accW1[FT][ET];
#pragma unroll
    for (int o = 0; o < HET; ++o)
#pragma unroll
      for (int i = 0; i < ET; ++i) accM[o][i] = zero4();
#pragma unroll
    for (int o = 0; o < FT; ++o)
#pragma unroll
      for (int i = 0; i < ET; ++i) accW1[o][i] = zero4();
#pragma unroll 2
    for (int64_t t = t0; t < t1; t += STEP) {
      bool ok;  // false only for the missing second tile of an odd range (bf16)
      const TT* p = lane_ptr(t, ok);
      dw_pair<HET, ET>(accM, p, ok, R::GU, R::X);
      dw_pair<FT, ET>(accW1, p, ok, R::GF1, R::Y);
    }
    dw_tiles_store<HET, ET>(slab + a.G.M[d], E, accM);
    dw_tiles_store<FT, ET>(slab + a.G.W1[d], E, accW1);
  } else {  // N (gres ⊗ z) and W2 (gr2 ⊗ f1r)
    f4 accN[ET][HET], accW2[ET][FT];
#pragma unroll
    for (int o = 0; o < ET; ++o) {
#pragma unroll
      for (int i = 0; i < HET; ++i) accN[o][i] = zero4();
#pragma unroll
      for (int i = 0; i < FT; ++i) accW2[o][i] = zero4();
    }
#pragma unroll 2
    for (int64_t t = t0; t < t1; t += STEP) {
      bool ok;
      const TT* p = lane_ptr(t, ok);
      dw_pair<ET, HET>(accN, p, ok, R::GRES, R::Z);
      dw_pair<ET, FT>(accW2, p, ok, R::GR2, R::F1R);
    }
    dw_tiles_store<ET, HET>(slab + a.G.N[d], H * E, accN);
    dw_tiles_store<ET, FT>(slab + a.G.W2[d], FF, accW2);
  }
}

template <int E, int H, int FF, typename TT>
int launch_dw_gemm(int kind, const void* tape, int64_t ntiles, int D, float* slabs, int64_t slab_stride,
                   const t2o_layout& G, int nslab, hipStream_t stream) {
  if (D < 1 || D > T2O_MAX_DEPTH || nslab < 1) return T2O_EINVAL;
  DwGemmArgs a{};
  a.tape = tape;
  a.ntiles = ntiles;
  a.chunk = ((ntiles + nslab - 1) / nslab + 1) / 2 * 2;
  a.slabs = slabs;
  a.slab_stride = slab_stride;
  a.G = G;
  a.D = D;
  auto kern = kind == 0 ? dw_gemm_kernel<E, H, FF, 0, TT> : dw_gemm_kernel<E, H, FF, 1, TT>;
  hipLaunchKernelGGL(kern, dim3(nslab), dim3(64 * 2 * D), 0, stream, a);
  return (int)hipGetLastError();
}

}  // namespace t2o

using namespace t2o;

extern "C" int64_t t2o_bwd_tape_floats(const t2o_layout* L, int64_t tiles) {
  if (!L || tiles < 0) return -1;
  const int64_t elems = (int64_t)L->D * tiles * 16 * (4 * L->E + 2 * L->H * L->E + 2 * L->FF);
  return L->prec ? (elems + 1) / 2 : elems;
}

extern "C" int t2o_bwd_tape_contract(const t2o_layout* L, const void* tape, int64_t tiles, float* gslabs,
                                     int nslab, void* stream) {
  if (!L || !tape || !gslabs || tiles < 0 || nslab < 1) return T2O_EINVAL;
  t2o_layout G;
  grad_layout(*L, G);
  int rc = T2O_EUNSUPPORTED;
  T2O_DISPATCH(L->E, L->H, L->D, L->n_ent, L->FF,
               rc = (L->prec ? launch_dw_gemm<E_, H_, FF_, __bf16>(L->kind, tape, tiles, L->D, gslabs, G.grad_total,
                                                                  G, nslab, (hipStream_t)stream)
                             : launch_dw_gemm<E_, H_, FF_, float>(L->kind, tape, tiles, L->D, gslabs, G.grad_total,
                                                                 G, nslab, (hipStream_t)stream)));
  return rc;
}
