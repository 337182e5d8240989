// t2o_dwgemm.hip — contraction of the weight-gradient tape (TapeRec, t2o_common.hpp).
//
// dM = Σ_n gu_n x_nᵀ,  dN = Σ_n gres_n z_nᵀ,  dW1 = Σ_n gf1_n y_nᵀ,  dW2 = Σ_n gr2_n f1r_nᵀ
// over every record n (row x step of the agent, query row x step of the mixer)
// of every block.  This is a tall-skinny GEMM with K = records: split-K over
// workgroups (workgroup k contracts one contiguous record range and writes the
// four matrices of every block into gradient slab k, whose small-gradient part
// the backward kernel has already filled), and inside a workgroup one wave per
// (block, matrix pair) keeps its 28 output tiles in MFMA accumulators for the
// whole range.  MFMA step: lane (g, c) feeds record n0+g — A = dY[n0+g][16o+c],
// B = X[n0+g][16i+c] — so each 16x16x4 MFMA adds four records.
// Bound: HBM (each record is read once: 2304 B per block at E=32, H=3, FF=128).
// Called by the host right after t2o_agent_unroll_bwd / t2o_mixer_unroll_bwd
// with the same slabs: it fills their M/N/W1/W2 regions.
#include "t2o_common.hpp"
#include "t2o_dispatch.hpp"
#include "t2o_layout.hpp"

namespace t2o {

struct DwGemmArgs {
  const float* tape;   // [D][nrec][TapeRec::SIZE]
  int64_t nrec;        // records per block
  int64_t chunk;       // records per workgroup (multiple of 4)
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

// one operand pair: acc[o][i] += Σ_{4 records} A[o-tile] ⊗ B[i-tile]
template <int OT, int IT>
T2O_DEV void dw_pair_step(f4 (&acc)[OT][IT], const float* __restrict__ rp, bool ok, int offA, int offB) {
  const int c = lane_c();
  float a[OT], b[IT];
#pragma unroll
  for (int o = 0; o < OT; ++o) a[o] = ok ? rp[offA + 16 * o + c] : 0.f;
#pragma unroll
  for (int i = 0; i < IT; ++i) b[i] = ok ? rp[offB + 16 * i + c] : 0.f;
#pragma unroll
  for (int o = 0; o < OT; ++o)
#pragma unroll
    for (int i = 0; i < IT; ++i) acc[o][i] = mfma4(a[o], b[i], acc[o][i]);
}

// KIND (0 agent, 1 mixer) only separates the two instances in profiles.
template <int E, int H, int FF, int KIND>
__global__ __launch_bounds__(64 * 2 * T2O_MAX_DEPTH) void dw_gemm_kernel(DwGemmArgs a) {
  using R = TapeRec<E, H, FF>;
  constexpr int ET = E / 16, HET = H * ET, FT = FF / 16;
  const int w = wave_id();
  const int d = w >> 1;
  if (d >= a.D) return;
  const int g = lane_g();
  const int64_t n0 = (int64_t)blockIdx.x * a.chunk;
  const int64_t n1 = n0 + a.chunk < a.nrec ? n0 + a.chunk : a.nrec;
  const float* __restrict__ base = a.tape + (size_t)d * a.nrec * R::SIZE;
  float* slab = a.slabs + (size_t)blockIdx.x * a.slab_stride;
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
    for (int64_t n = n0; n < n1; n += 4) {
      const int64_t nr = n + g;
      const bool ok = nr < n1;
      const float* rp = base + (ok ? nr : n0) * R::SIZE;
      dw_pair_step<HET, ET>(accM, rp, ok, R::GU, R::X);
      dw_pair_step<FT, ET>(accW1, rp, ok, R::GF1, R::Y);
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
    for (int64_t n = n0; n < n1; n += 4) {
      const int64_t nr = n + g;
      const bool ok = nr < n1;
      const float* rp = base + (ok ? nr : n0) * R::SIZE;
      dw_pair_step<ET, HET>(accN, rp, ok, R::GRES, R::Z);
      dw_pair_step<ET, FT>(accW2, rp, ok, R::GR2, R::F1R);
    }
    dw_tiles_store<ET, HET>(slab + a.G.N[d], H * E, accN);
    dw_tiles_store<ET, FT>(slab + a.G.W2[d], FF, accW2);
  }
}

template <int E, int H, int FF>
int launch_dw_gemm(int kind, const float* tape, int64_t nrec, int D, float* slabs, int64_t slab_stride, const t2o_layout& G,
                   int nslab, hipStream_t stream) {
  if (D < 1 || D > T2O_MAX_DEPTH || nslab < 1) return T2O_EINVAL;
  DwGemmArgs a{};
  a.tape = tape;
  a.nrec = nrec;
  a.chunk = ((nrec + nslab - 1) / nslab + 3) / 4 * 4;
  a.slabs = slabs;
  a.slab_stride = slab_stride;
  a.G = G;
  a.D = D;
  auto kern = kind == 0 ? dw_gemm_kernel<E, H, FF, 0> : dw_gemm_kernel<E, H, FF, 1>;
  hipLaunchKernelGGL(kern, dim3(nslab), dim3(64 * 2 * D), 0, stream, a);
  return (int)hipGetLastError();
}

}  // namespace t2o

using namespace t2o;

extern "C" int64_t t2o_bwd_tape_floats(const t2o_layout* L, int64_t records) {
  if (!L || records < 0) return -1;
  return (int64_t)L->D * records * (4 * L->E + 2 * L->H * L->E + 2 * L->FF);
}

extern "C" int t2o_bwd_tape_contract(const t2o_layout* L, const float* tape, int64_t records, float* gslabs,
                                     int nslab, void* stream) {
  if (!L || !tape || !gslabs || records < 0 || nslab < 1) return T2O_EINVAL;
  t2o_layout G;
  grad_layout(*L, G);
  int rc = T2O_EUNSUPPORTED;
  T2O_DISPATCH(L->E, L->H, L->D, L->n_ent, L->FF,
               rc = (launch_dw_gemm<E_, H_, FF_>(L->kind, tape, records, L->D, gslabs, G.grad_total, G, nslab,
                                                 (hipStream_t)stream)));
  return rc;
}
