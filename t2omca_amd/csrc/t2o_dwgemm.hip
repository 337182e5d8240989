// t2o_dwgemm.hip — contraction of the weight-gradient tape (TapeRec, t2o_common.hpp).
//
// Per block d, over every record n (row x step of the agent, query row x step
// of the mixer):
//   dM  = Σ_n gu_n ⊗ x_n          dN  = Σ_n gres_n ⊗ z_n
//   dW2 = Σ_n gr2_n ⊗ relu(f1_n)  dW1 = Σ_n gf1_n ⊗ y_n
// where f1 = W1 y + c1 and gf1 = [f1 > 0] ⊙ (W2ᵀ gr2) are recomputed here from
// the record's (y, gr2) — the backward kernels do not store them.
//
// This is a tall-skinny GEMM with K = records (≈1M per block at config 3) and
// HBM-bound: every tape byte is read once.  Structure:
//   * split-K over workgroups: 16-record tiles are grouped TG at a time and the
//     groups dealt round-robin (group k -> workgroup k mod nslab), so the grid
//     streams one contiguous window of the tape at a time; workgroup k writes
//     the four matrices of every block into gradient slab k, whose small-
//     gradient part the backward kernel has already filled;
//   * each workgroup stages a group (all D blocks) in LDS with full-line 16-B
//     loads by all its threads, double-buffered in LDS with a two-deep
//     register ring (prefetch distance two groups), one barrier per group;
//   * 4 waves per block read the staged tiles: wave 0 dM, wave 1 dN, waves 2
//     and 3 one half of the FF features each (recompute f1 / gf1 with MFMA
//     from LDS copies of W1 / W2ᵀ, then dW1 / dW2).  All accumulators stay in
//     registers for the whole launch.
// MFMA shapes: bf16 tape -> v_mfma_f32_16x16x16_bf16 (K = 16 records of a
// tile: lane (g, c) reads records 4g..4g+3 of one feature, one ds_read_b64;
// the record-major operand of the recompute comes from ds_read_b64_tr_b16);
// fp32 tape -> four v_mfma_f32_16x16x4_f32 per 16 records.
#include <type_traits>

#include "t2o_common.hpp"
#include "t2o_dispatch.hpp"
#include "t2o_layout.hpp"

namespace t2o {

struct DwGemmArgs {
  const void* tape;    // [D][ntiles][SIZE][16]
  int64_t ntiles;      // 16-record tiles per block
  float* slabs;        // [nslab][slab_stride], compact gradient layout G
  int64_t slab_stride;
  const float* pack;   // the network's kernel pack (fp32; bf16 image at pack + L.total)
  t2o_layout L, G;
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

typedef uint32_t u4v __attribute__((ext_vector_type(4)));

template <typename TT> struct DwTraits;
template <> struct DwTraits<__bf16> { static constexpr int TG = 2; };  // tiles per group
template <> struct DwTraits<float> { static constexpr int TG = 1; };

// ---- operand reads from a staged tile (feature-major, 16 records per row) ----
// bf16: records 4g..4g+3 of feature row `f` (K-slice of a 16x16x16 MFMA)
T2O_DEV bf4 kslice(const __bf16* tile, int f) { return ldb4(tile + f * 16 + 4 * lane_g()); }
// bf16: features f0 + 4g .. +3 of record c (the record-major operand), by the
// gfx950 transposed LDS read: lane 4q+p of each 16-lane group addresses row
// f0 + 4g + q, records 4p..4p+3, and lane c receives record c of the 4 rows.
T2O_DEV bf4 rslice(const __bf16* tile, int f0) {
  const int c = lane_c();
  const __bf16* p = tile + (f0 + 4 * lane_g() + (c >> 2)) * 16 + 4 * (c & 3);
  typedef __attribute__((address_space(3))) s4v lds_s4v;
  const s4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(p));
  return __builtin_bit_cast(bf4, v);
}

template <int E, int H, int FF, int D, typename TT>
struct DwDims {
  using R = TapeRec<E, H, FF>;
  static constexpr int ET = E / 16, HET = H * ET, FT = FF / 16, FH = FT / 2;
  static constexpr bool BF = sizeof(TT) == 2;
  static constexpr int TG = DwTraits<TT>::TG;
  static constexpr int TILE = R::SIZE * 16;                 // elements per tile
  static constexpr int CPT = TILE * (int)sizeof(TT) / 16;   // 16-B chunks per tile
  static constexpr int NT = 256 * D;                        // threads
  static constexpr int GCH = D * TG * CPT;                  // chunks per group
  static constexpr int NLD = (GCH + NT - 1) / NT;           // chunks per thread
  static constexpr int GELEM = D * TG * TILE;               // elements per staged group
  static_assert(FT % 2 == 0, "FF must split into two halves of 16-feature tiles");
};

// group j of this workgroup: tape -> registers (tiles past the end read as zeros)
template <typename Dm, typename TT>
T2O_DEV void dw_load(const DwGemmArgs& a, int64_t j, u4v (&rg)[Dm::NLD]) {
  const TT* __restrict__ tape = static_cast<const TT*>(a.tape);
  const int64_t grp = blockIdx.x + j * gridDim.x;
#pragma unroll
  for (int i = 0; i < Dm::NLD; ++i) {
    const int q = threadIdx.x + i * Dm::NT;
    const int dd = q / (Dm::TG * Dm::CPT), rem = q % (Dm::TG * Dm::CPT);
    const int tt = rem / Dm::CPT, ch = rem % Dm::CPT;
    const int64_t tile = grp * Dm::TG + tt;
    rg[i] = u4v{0u, 0u, 0u, 0u};
    if (q < Dm::GCH && tile < a.ntiles)
      rg[i] = *reinterpret_cast<const u4v*>(tape + ((size_t)dd * a.ntiles + tile) * Dm::TILE + ch * (16 / sizeof(TT)));
  }
}
// registers -> LDS group buffer (lane-linear: the buffer is [D][TG][tile])
template <typename Dm, typename TT>
T2O_DEV void dw_store(TT* buf, const u4v (&rg)[Dm::NLD]) {
#pragma unroll
  for (int i = 0; i < Dm::NLD; ++i) {
    const int q = threadIdx.x + i * Dm::NT;
    if (q < Dm::GCH) *reinterpret_cast<u4v*>(buf + q * (16 / sizeof(TT))) = rg[i];
  }
}

// Role state: the accumulators (and, for the FFN roles, the weight fragments)
// of one wave.  ROLE 0 dM, 1 dN, 2/3 FFN half 0/1.
template <int ROLE, int E, int H, int FF, int D, typename TT>
struct DwRole;

template <int E, int H, int FF, int D, typename TT>
struct DwRole<0, E, H, FF, D, TT> {
  using Dm = DwDims<E, H, FF, D, TT>;
  using R = typename Dm::R;
  f4 acc[Dm::HET][Dm::ET];  // dM[gu feature][x feature]
  T2O_DEV void init(const DwGemmArgs&, int, const TT*) {
#pragma unroll
    for (int o = 0; o < Dm::HET; ++o)
#pragma unroll
      for (int i = 0; i < Dm::ET; ++i) acc[o][i] = zero4();
  }
  T2O_DEV void tile(const TT* t) {
    const int c = lane_c(), g = lane_g();
    if constexpr (Dm::BF) {
      bf4 xb[Dm::ET];
#pragma unroll
      for (int i = 0; i < Dm::ET; ++i) xb[i] = kslice(t, R::X + 16 * i + c);
#pragma unroll
      for (int o = 0; o < Dm::HET; ++o) {
        const bf4 ab = kslice(t, R::GU + 16 * o + c);
#pragma unroll
        for (int i = 0; i < Dm::ET; ++i) acc[o][i] = mfma_b16(ab, xb[i], acc[o][i]);
      }
    } else {
      f4 xv[Dm::ET];
#pragma unroll
      for (int i = 0; i < Dm::ET; ++i) xv[i] = ld4(t + (R::X + 16 * i + c) * 16 + 4 * g);
#pragma unroll
      for (int o = 0; o < Dm::HET; ++o) {
        const f4 av = ld4(t + (R::GU + 16 * o + c) * 16 + 4 * g);
#pragma unroll
        for (int i = 0; i < Dm::ET; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[o][i] = mfma4(av[r], xv[i][r], acc[o][i]);
      }
    }
  }
  T2O_DEV void finish(const DwGemmArgs& a, float* slab, int d) {
    dw_tiles_store<Dm::HET, Dm::ET>(slab + a.G.M[d], E, acc);
  }
};

template <int E, int H, int FF, int D, typename TT>
struct DwRole<1, E, H, FF, D, TT> {
  using Dm = DwDims<E, H, FF, D, TT>;
  using R = typename Dm::R;
  f4 acc[Dm::ET][Dm::HET];  // dN[gres feature][z feature]
  T2O_DEV void init(const DwGemmArgs&, int, const TT*) {
#pragma unroll
    for (int o = 0; o < Dm::ET; ++o)
#pragma unroll
      for (int i = 0; i < Dm::HET; ++i) acc[o][i] = zero4();
  }
  T2O_DEV void tile(const TT* t) {
    const int c = lane_c(), g = lane_g();
    if constexpr (Dm::BF) {
      bf4 gb[Dm::ET];
#pragma unroll
      for (int o = 0; o < Dm::ET; ++o) gb[o] = kslice(t, R::GRES + 16 * o + c);
#pragma unroll
      for (int i = 0; i < Dm::HET; ++i) {
        const bf4 zb = kslice(t, R::Z + 16 * i + c);
#pragma unroll
        for (int o = 0; o < Dm::ET; ++o) acc[o][i] = mfma_b16(gb[o], zb, acc[o][i]);
      }
    } else {
      f4 gv[Dm::ET];
#pragma unroll
      for (int o = 0; o < Dm::ET; ++o) gv[o] = ld4(t + (R::GRES + 16 * o + c) * 16 + 4 * g);
#pragma unroll
      for (int i = 0; i < Dm::HET; ++i) {
        const f4 zv = ld4(t + (R::Z + 16 * i + c) * 16 + 4 * g);
#pragma unroll
        for (int o = 0; o < Dm::ET; ++o)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[o][i] = mfma4(gv[o][r], zv[r], acc[o][i]);
      }
    }
  }
  T2O_DEV void finish(const DwGemmArgs& a, float* slab, int d) {
    dw_tiles_store<Dm::ET, Dm::HET>(slab + a.G.N[d], H * E, acc);
  }
};

// FFN half HALF: recompute f1 = W1 y + c1 and gf1 = [f1 > 0] ⊙ W2ᵀ gr2 for the
// half's FH feature tiles as [records x features] MFMA tiles (lane (g, c) =
// records 4g..4g+3 of feature 16J + c — already the K-slice layout of the
// contraction), then dW2[e][J] += gr2 ⊗ relu(f1), dW1[J][e] += gf1 ⊗ y.
template <int HALF, int E, int H, int FF, int D, typename TT>
struct DwFfn {
  using Dm = DwDims<E, H, FF, D, TT>;
  using R = typename Dm::R;
  static constexpr int ET = Dm::ET, FH = Dm::FH;
  using Frag = typename std::conditional<Dm::BF, bf4, f4>::type;
  f4 acc1[FH][ET];  // dW1 rows of this half
  f4 acc2[ET][FH];  // dW2 columns of this half
  const TT* wl;    // LDS copy of this block's W1 [FF][E] then W2ᵀ [FF][E] (bf16: the pack's swizzled image)
  float c1v[FH];
  T2O_DEV void init(const DwGemmArgs& a, int d, const TT* wlds) {
    const int c = lane_c();
#pragma unroll
    for (int o = 0; o < FH; ++o)
#pragma unroll
      for (int i = 0; i < ET; ++i) acc1[o][i] = acc2[i][o] = zero4();
    wl = wlds + (size_t)d * 2 * FF * E;
#pragma unroll
    for (int jt = 0; jt < FH; ++jt) c1v[jt] = a.pack[a.L.c1[d] + 16 * (HALF * FH + jt) + c];
  }
  // fragment of W (0: W1, 1: W2ᵀ): row 16J + c, features 16s + 4g .. +3
  T2O_DEV Frag wfrag(int m, int jt, int s) const {
    const int row = 16 * (HALF * FH + jt) + lane_c();
    const TT* base = wl + (size_t)m * FF * E + (size_t)row * E;
    if constexpr (Dm::BF) return ldb4(base + ((16 * s + 4 * lane_g()) ^ bf_swz(row, E)));
    else return ld4(base + 16 * s + 4 * lane_g());
  }
  T2O_DEV void tile(const TT* t) {
    const int c = lane_c(), g = lane_g();
    if constexpr (Dm::BF) {
      bf4 yr[ET], gr[ET], yk[ET], gk[ET];
#pragma unroll
      for (int s = 0; s < ET; ++s) {
        yr[s] = rslice(t, R::Y + 16 * s);
        gr[s] = rslice(t, R::GR2 + 16 * s);
        yk[s] = kslice(t, R::Y + 16 * s + c);
        gk[s] = kslice(t, R::GR2 + 16 * s + c);
      }
#pragma unroll
      for (int jt = 0; jt < FH; ++jt) {
        f4 f1 = zero4(), gp = zero4();
#pragma unroll
        for (int s = 0; s < ET; ++s) {
          f1 = mfma_b16(yr[s], wfrag(0, jt, s), f1);
          gp = mfma_b16(gr[s], wfrag(1, jt, s), gp);
        }
        f4 fr, gf;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = f1[r] + c1v[jt];
          fr[r] = fmaxf(v, 0.f);
          gf[r] = v > 0.f ? gp[r] : 0.f;
        }
        const bf4 frb = to_bf4(fr), gfb = to_bf4(gf);
#pragma unroll
        for (int e = 0; e < ET; ++e) {
          acc2[e][jt] = mfma_b16(gk[e], frb, acc2[e][jt]);
          acc1[jt][e] = mfma_b16(gfb, yk[e], acc1[jt][e]);
        }
      }
    } else {
      f4 yk[ET], gk[ET];
#pragma unroll
      for (int s = 0; s < ET; ++s) {
        yk[s] = ld4(t + (R::Y + 16 * s + c) * 16 + 4 * g);
        gk[s] = ld4(t + (R::GR2 + 16 * s + c) * 16 + 4 * g);
      }
#pragma unroll
      for (int jt = 0; jt < FH; ++jt) {
        f4 f1 = zero4(), gp = zero4();
#pragma unroll
        for (int s = 0; s < ET; ++s) {
          const f4 w1 = wfrag(0, jt, s), w2 = wfrag(1, jt, s);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // feature k = 16s + 4g + r of record c (K-step r, k index g)
            const int fk = 16 * s + 4 * g + r;
            f1 = mfma4(t[(R::Y + fk) * 16 + c], w1[r], f1);
            gp = mfma4(t[(R::GR2 + fk) * 16 + c], w2[r], gp);
          }
        }
        f4 fr, gf;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = f1[r] + c1v[jt];
          fr[r] = fmaxf(v, 0.f);
          gf[r] = v > 0.f ? gp[r] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < ET; ++e)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc2[e][jt] = mfma4(gk[e][r], fr[r], acc2[e][jt]);
            acc1[jt][e] = mfma4(gf[r], yk[e][r], acc1[jt][e]);
          }
      }
    }
  }
  T2O_DEV void finish(const DwGemmArgs& a, float* slab, int d) {
    dw_tiles_store<FH, ET>(slab + a.G.W1[d] + (int64_t)16 * HALF * FH * E, E, acc1);
    dw_tiles_store<ET, FH>(slab + a.G.W2[d] + 16 * HALF * FH, FF, acc2);
  }
};
template <int E, int H, int FF, int D, typename TT>
struct DwRole<2, E, H, FF, D, TT> : DwFfn<0, E, H, FF, D, TT> {};
template <int E, int H, int FF, int D, typename TT>
struct DwRole<3, E, H, FF, D, TT> : DwFfn<1, E, H, FF, D, TT> {};

// One wave's whole launch for its role (every role runs the same pipeline and
// the same barrier sequence; the roles only differ in what they read).
// Pipeline: LDS double buffer, register ring of two, prefetch distance 2.
template <int ROLE, int E, int H, int FF, int D, typename TT>
T2O_DEV void dw_run(const DwGemmArgs& a, TT* buf0, TT* buf1, const TT* wlds, int d) {
  using Dm = DwDims<E, H, FF, D, TT>;
  const int64_t ngroups = (a.ntiles + Dm::TG - 1) / Dm::TG;
  const int64_t nj = (int64_t)blockIdx.x < ngroups ? (ngroups - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  DwRole<ROLE, E, H, FF, D, TT> st;
  st.init(a, d, wlds);
  auto compute = [&](const TT* buf) {
#pragma unroll
    for (int tt = 0; tt < Dm::TG; ++tt) {
      st.tile(buf + (d * Dm::TG + tt) * Dm::TILE);
      T2O_FENCE();  // keep the next tile's LDS reads from being hoisted over these MFMAs
    }
  };
  u4v r0[Dm::NLD], r1[Dm::NLD];
  if (nj > 0) dw_load<Dm, TT>(a, 0, r0);
  if (nj > 1) dw_load<Dm, TT>(a, 1, r1);
  if (nj > 0) dw_store<Dm, TT>(buf0, r0);
  if (nj > 1) dw_store<Dm, TT>(buf1, r1);
  if (nj > 2) dw_load<Dm, TT>(a, 2, r0);
  if (nj > 3) dw_load<Dm, TT>(a, 3, r1);
  __syncthreads();
  for (int64_t j = 0; j < nj; j += 2) {
    compute(buf0);
    __syncthreads();
    if (j + 2 < nj) dw_store<Dm, TT>(buf0, r0);
    if (j + 4 < nj) dw_load<Dm, TT>(a, j + 4, r0);
    if (j + 1 >= nj) break;
    compute(buf1);
    __syncthreads();
    if (j + 3 < nj) dw_store<Dm, TT>(buf1, r1);
    if (j + 5 < nj) dw_load<Dm, TT>(a, j + 5, r1);
  }
  st.finish(a, a.slabs + (size_t)blockIdx.x * a.slab_stride, d);
}

template <int E, int H, int FF, int D, int KIND, typename TT>
__global__ __launch_bounds__(256 * D) void dw_gemm_kernel(DwGemmArgs a) {
  using Dm = DwDims<E, H, FF, D, TT>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  TT* const buf0 = reinterpret_cast<TT*>(smem);
  TT* const buf1 = buf0 + Dm::GELEM;
  TT* const wlds = buf1 + Dm::GELEM;  // [D][W1, W2ᵀ][FF][E]
  {  // stage W1 / W2ᵀ of every block (made visible by dw_run's first barrier)
    const TT* img = Dm::BF ? reinterpret_cast<const TT*>(a.pack + a.L.total) : reinterpret_cast<const TT*>(a.pack);
    constexpr int PER = 16 / sizeof(TT), MAT = FF * E;
    for (int q = threadIdx.x; q < D * 2 * MAT / PER; q += Dm::NT) {
      const int e = q * PER, dd = e / (2 * MAT), m = (e / MAT) & 1, k = e % MAT;
      const int64_t src = (m ? a.L.W2T[dd] : a.L.W1[dd]) + k;
      *reinterpret_cast<u4v*>(wlds + e) = *reinterpret_cast<const u4v*>(img + src);
    }
  }
  const int w = wave_id();
  const int d = w >> 2, role = w & 3;
  switch (role) {  // wave-uniform; the four paths issue the same barriers
    case 0: dw_run<0, E, H, FF, D, TT>(a, buf0, buf1, wlds, d); break;
    case 1: dw_run<1, E, H, FF, D, TT>(a, buf0, buf1, wlds, d); break;
    case 2: dw_run<2, E, H, FF, D, TT>(a, buf0, buf1, wlds, d); break;
    default: dw_run<3, E, H, FF, D, TT>(a, buf0, buf1, wlds, d); break;
  }
}

template <int E, int H, int FF, int D, typename TT>
int launch_dw_gemm(int kind, const void* tape, int64_t ntiles, const float* pack, float* slabs, const t2o_layout& L,
                   const t2o_layout& G, int nslab, hipStream_t stream) {
  if (nslab < 1) return T2O_EINVAL;
  DwGemmArgs a{};
  a.tape = tape;
  a.ntiles = ntiles;
  a.slabs = slabs;
  a.slab_stride = G.grad_total;
  a.pack = pack;
  a.L = L;
  a.G = G;
  const size_t lds = sizeof(TT) * ((size_t)2 * D * DwTraits<TT>::TG * TapeRec<E, H, FF>::SIZE * 16 +
                                    (size_t)D * 2 * FF * E);
  auto kern = kind == 0 ? dw_gemm_kernel<E, H, FF, D, 0, TT> : dw_gemm_kernel<E, H, FF, D, 1, TT>;
  if (lds > 160 * 1024) return T2O_EUNSUPPORTED;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(nslab), dim3(256 * D), lds, stream, a);
  return (int)hipGetLastError();
}

}  // namespace t2o

using namespace t2o;

extern "C" int64_t t2o_bwd_tape_floats(const t2o_layout* L, int64_t tiles) {
  if (!L || tiles < 0) return -1;
  const int64_t elems = (int64_t)L->D * tiles * 16 * (4 * L->E + 2 * L->H * L->E);
  return L->prec ? (elems + 1) / 2 : elems;
}

extern "C" int t2o_bwd_tape_contract(const t2o_layout* L, const float* pack, const void* tape, int64_t tiles,
                                     float* gslabs, int nslab, void* stream) {
  if (!L || !pack || !tape || !gslabs || tiles < 0 || nslab < 1) return T2O_EINVAL;
  t2o_layout G;
  grad_layout(*L, G);
  int rc = T2O_EUNSUPPORTED;
  T2O_DISPATCH(L->E, L->H, L->D, L->n_ent, L->FF,
               rc = (L->prec ? launch_dw_gemm<E_, H_, FF_, D_, __bf16>(L->kind, tape, tiles, pack, gslabs, *L, G,
                                                                       nslab, (hipStream_t)stream)
                             : launch_dw_gemm<E_, H_, FF_, D_, float>(L->kind, tape, tiles, pack, gslabs, *L, G,
                                                                      nslab, (hipStream_t)stream)));
  return rc;
}
