// t2o_dwgemm.hip — contraction of the weight-gradient tape (TapeRec, t2o_common.hpp).
//
// Per block d, over every record n (row x step of the agent, query row x step
// of the mixer):
//   dM  = Σ_n gu_n ⊗ x_n          dN  = Σ_n gres_n ⊗ z_n
//   dW2 = Σ_n gr2_n ⊗ relu(f1_n)  P   = Σ_n gf1_n ⊗ x̂1_n
//   d bu = Σ gres,  d c2 = Σ gr2,  d c1 = Σ gf1,  Q = Σ gr2 ⊙ x̂1
// where y = x̂1 ⊙ g1 + n1, f1 = W1 y + c1 and gf1 = [f1 > 0] ⊙ (W2ᵀ gr2) are
// recomputed here from the record's (x̂1, gr2) — the backward kernels store
// neither y nor its grad.  P and Q go to the slab's W1 and g1 slots;
// t2o_unpack_grads turns them into dW1, d g1 and d n1 (TapeRec's comment).
//
// This is a tall-skinny GEMM with K = records (≈1M per block at config 3) and
// HBM-bound: every tape byte is read once.  Structure:
//   * split-K over workgroups: 16-record tiles are grouped TG at a time and the
//     groups dealt round-robin (group k -> workgroup k mod nslab), so the grid
//     streams one contiguous window of the tape at a time; workgroup k writes
//     its matrices and vectors of every block into gradient slab k, whose
//     other (small-gradient) part the backward kernel has already filled;
//   * each workgroup stages a group (all D blocks) in LDS with full-line 16-B
//     loads by all its threads (records padded in LDS so both read kinds below
//     are bank-conflict-free), double-buffered in LDS with a two-deep register
//     ring (prefetch distance two groups), one barrier per group;
//   * 4 waves per block read the staged tiles: wave 0 dM (+ Q), wave 1
//     dN (+ bu), waves 2 and 3 one half of the FF features each (recompute
//     y, f1 / gf1 with MFMA, then P / dW2 and c1; wave 2 also c2).  All
//     accumulators stay in registers for the whole launch.
// MFMA shapes: bf16 tape -> v_mfma_f32_16x16x16_bf16 with K = the 16 records
// of a tile.  The tape is record-major, so the feature-major K-slices (records
// 4g..4g+3 of one feature) come from ds_read_b64_tr_b16 and the record-major
// operand of the recompute (features 4g..4g+3 of record c) from a plain
// ds_read_b64.  fp32 tape -> four v_mfma_f32_16x16x4_f32 per 16 records.
#include <type_traits>

#include "t2o_common.hpp"
#include "t2o_dispatch.hpp"
#include "t2o_generic.hpp"
#include "t2o_layout.hpp"

namespace t2o {

struct DwGemmArgs {
  const void* tape;    // [D][ntiles][16][SIZE]
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

// per-lane partial sums of a vector over this lane's records (lane (g, c) =
// feature 16t + c): sum the 4 lane groups and write from group 0
template <int NT>
T2O_DEV void dw_vec_store(float* __restrict__ v, const float (&acc)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float s = allsum4(acc[t]);
    if (lane_g() == 0) v[16 * t + lane_c()] = s;
  }
}

typedef uint32_t u4v __attribute__((ext_vector_type(4)));

// bf16, the lean agent record: tiles are contracted in pairs (K = 32 records per
// 16x16x32 MFMA).  The full (mixer) record keeps one tile per 16x16x16 MFMA: its
// pair form needs 256 VGPRs plus 12 B of scratch, measured 14 us faster per update
// alone (profiles/r5_dwp/), and one of four round-5 suites on it failed the
// run-to-run reproducibility check (r5_final2; 87 later runs reproduced,
// profiles/r6_hunt/x3_stress_pf.log, the cause unnamed): removed in round 6.
template <typename TT> struct DwTraits;
template <> struct DwTraits<__bf16> { static constexpr int TG = 2, PADC = 2; };  // tiles per group, pad chunks
template <> struct DwTraits<float> { static constexpr int TG = 1, PADC = 1; };

// FMT 0: the full record (TapeRec); 1: the lean agent record (TapeRecA: dM and
// dN were accumulated by the BPTT kernel, roles 0 / 1 keep only their vectors)
template <int E, int H, int FF, int D, typename TT, int RT = 16, int FMT = 0>
struct DwDims {
  using R = typename std::conditional<FMT == 1, TapeRecA<E, H, FF>, TapeRec<E, H, FF>>::type;
  static constexpr bool MN = R::GU >= 0;  // dM / dN operands on the tape
  static constexpr int ET = E / 16, HET = H * ET, FT = FF / 16, FH = FT / 2;
  static constexpr bool BF = sizeof(TT) == 2;
  // tiles per group: the lean agent record is a third of the full one, so its
  // groups take more tiles (the same bytes in flight per workgroup)
  static constexpr int TG = (FMT == 1 && BF) ? 4 : DwTraits<TT>::TG;
  static constexpr int PER = 16 / (int)sizeof(TT);          // elements per 16-B chunk
  static constexpr int CPR = R::SIZE / PER;                  // chunks per record
  static constexpr int CPT = RT * CPR;                       // chunks per tile (HBM: RT records)
  static constexpr int RSTR = (CPR + DwTraits<TT>::PADC) * PER;  // padded LDS record stride (elements)
  static constexpr int TSTR = 16 * RSTR;                     // LDS tile stride (elements)
  static constexpr int NT = 256 * D;                         // threads
  static constexpr int GCH = D * TG * CPT;                   // chunks per group
  static constexpr int NLD = (GCH + NT - 1) / NT;            // chunks per thread
  static constexpr int GELEM = D * TG * TSTR;                // LDS elements per staged group
  static_assert(R::SIZE % PER == 0, "record must be a whole number of 16-B chunks");
  static_assert(FT % 2 == 0, "FF must split into two halves of 16-feature tiles");
};

// group j of this workgroup: tape -> registers (tiles past the end read as zeros)
template <typename Dm, typename TT>
T2O_DEV void dw_load(const DwGemmArgs& a, int wg, int nwg, int64_t j, u4v (&rg)[Dm::NLD]) {
  const TT* __restrict__ tape = static_cast<const TT*>(a.tape);
  const int64_t grp = wg + j * nwg;
#pragma unroll
  for (int i = 0; i < Dm::NLD; ++i) {
    const int q = threadIdx.x + i * Dm::NT;
    const int dd = q / (Dm::TG * Dm::CPT), rem = q % (Dm::TG * Dm::CPT);
    const int tt = rem / Dm::CPT, ch = rem % Dm::CPT;
    const int64_t tile = grp * Dm::TG + tt;
    rg[i] = u4v{0u, 0u, 0u, 0u};
    if (q < Dm::GCH && tile < a.ntiles)
      rg[i] = *reinterpret_cast<const u4v*>(tape + ((size_t)dd * a.ntiles + tile) * Dm::CPT * Dm::PER +
                                            (size_t)ch * Dm::PER);
  }
}
// registers -> LDS group buffer [D][TG][16 records, padded stride RSTR]
template <typename Dm, typename TT>
T2O_DEV void dw_store(TT* buf, const u4v (&rg)[Dm::NLD]) {
#pragma unroll
  for (int i = 0; i < Dm::NLD; ++i) {
    const int q = threadIdx.x + i * Dm::NT;
    if (q < Dm::GCH) {
      const int tix = q / Dm::CPT, ch = q % Dm::CPT;  // tix = dd * TG + tt
      const int rec = ch / Dm::CPR, cr = ch % Dm::CPR;
      *reinterpret_cast<u4v*>(buf + tix * Dm::TSTR + rec * Dm::RSTR + cr * Dm::PER) = rg[i];
    }
  }
}

// ---- operand reads from a staged tile (record-major, stride RSTR) -----------
// K-slice: records 4g..4g+3 of feature f0 + c.  bf16 by the gfx950 transposed
// LDS read: lane 4q+p of each 16-lane group addresses record 4g + q, features
// f0 + 4p .. +3, and lane c receives feature f0 + c of the 4 records.
template <int RSTR>
T2O_DEV bf4 kslice(const __bf16* tile, int f0) {
  const int c = lane_c();
  const __bf16* p = tile + (4 * lane_g() + (c >> 2)) * RSTR + f0 + 4 * (c & 3);
  typedef __attribute__((address_space(3))) s4v lds_s4v;
  const s4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(p));
  return __builtin_bit_cast(bf4, v);
}
template <int RSTR>
T2O_DEV f4 kslice(const float* tile, int f0) {
  const int c = lane_c(), g = lane_g();
  f4 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = tile[(4 * g + r) * RSTR + f0 + c];
  return v;
}
// record-major operand: features f0 + 4g .. +3 of record c
template <int RSTR>
T2O_DEV bf4 rslice(const __bf16* tile, int f0) { return ldb4(tile + lane_c() * RSTR + f0 + 4 * lane_g()); }
template <int RSTR>
T2O_DEV f4 rslice(const float* tile, int f0) { return ld4(tile + lane_c() * RSTR + f0 + 4 * lane_g()); }

T2O_DEV float bsum4(bf4 v) { return ((float)v[0] + (float)v[1]) + ((float)v[2] + (float)v[3]); }
T2O_DEV float bsum4(f4 v) { return (v[0] + v[1]) + (v[2] + v[3]); }
T2O_DEV float bdot4(bf4 a, bf4 b) {
  return ((float)a[0] * (float)b[0] + (float)a[1] * (float)b[1]) + ((float)a[2] * (float)b[2] + (float)a[3] * (float)b[3]);
}
T2O_DEV float bdot4(f4 a, f4 b) { return (a[0] * b[0] + a[1] * b[1]) + (a[2] * b[2] + a[3] * b[3]); }

// two bf16 slices as one 16x16x32 operand (K = the first's 4 values, then the second's)
T2O_DEV bf8 cat8(bf4 a, bf4 b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7); }
T2O_DEV f4 kmma8(bf8 a, bf8 b, f4 acc) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0); }

// acc += A-slice ⊗ B-slice over the tile's 16 records (K-slices as above)
T2O_DEV f4 kmma(bf4 a, bf4 b, f4 acc) { return mfma_b16(a, b, acc); }
T2O_DEV f4 kmma(f4 a, f4 b, f4 acc) {
#pragma unroll
  for (int r = 0; r < 4; ++r) acc = mfma4(a[r], b[r], acc);
  return acc;
}

// Role state: the accumulators of one wave.  ROLE 0 dM (+ Q), 1 dN (+ bu),
// 2/3 FFN half 0/1 (+ c1 of the half; role 2 also c2).
template <int ROLE, int E, int H, int FF, int D, typename TT, int FMT>
struct DwRole;

template <int E, int H, int FF, int D, typename TT, int FMT>
struct DwRole<0, E, H, FF, D, TT, FMT> {
  using Dm = DwDims<E, H, FF, D, TT, 16, FMT>;
  using R = typename Dm::R;
  using Frag = typename std::conditional<Dm::BF, bf4, f4>::type;
  f4 acc[Dm::HET][Dm::ET];  // dM[gu feature][x feature]
  float vq[Dm::ET];         // Q = Σ gr2 ⊙ x̂1
  T2O_DEV void ready() {}
  T2O_DEV void init(const DwGemmArgs&, int, const TT*) {
#pragma unroll
    for (int o = 0; o < Dm::HET; ++o)
#pragma unroll
      for (int i = 0; i < Dm::ET; ++i) acc[o][i] = zero4();
#pragma unroll
    for (int i = 0; i < Dm::ET; ++i) vq[i] = 0.f;
  }
  T2O_DEV void tile(const TT* t) {
    constexpr int S = Dm::RSTR;
    if constexpr (Dm::MN) {
      Frag xb[Dm::ET];
#pragma unroll
      for (int i = 0; i < Dm::ET; ++i) xb[i] = kslice<S>(t, R::X + 16 * i);
#pragma unroll
      for (int o = 0; o < Dm::HET; ++o) {
        const Frag ab = kslice<S>(t, R::GU + 16 * o);
#pragma unroll
        for (int i = 0; i < Dm::ET; ++i) acc[o][i] = kmma(ab, xb[i], acc[o][i]);
      }
    }
#pragma unroll
    for (int i = 0; i < Dm::ET; ++i) vq[i] += bdot4(kslice<S>(t, R::GR2 + 16 * i), kslice<S>(t, R::XH1 + 16 * i));
  }
  // bf16, two tiles at once: K = their 32 records, one 16x16x32 MFMA per product
  T2O_DEV void tile2(const TT* ta, const TT* tb) {
    constexpr int S = Dm::RSTR;
    if constexpr (Dm::MN) {
      bf8 xb[Dm::ET];
#pragma unroll
      for (int i = 0; i < Dm::ET; ++i) xb[i] = cat8(kslice<S>(ta, R::X + 16 * i), kslice<S>(tb, R::X + 16 * i));
#pragma unroll
      for (int o = 0; o < Dm::HET; ++o) {
        const bf8 ab = cat8(kslice<S>(ta, R::GU + 16 * o), kslice<S>(tb, R::GU + 16 * o));
#pragma unroll
        for (int i = 0; i < Dm::ET; ++i) acc[o][i] = kmma8(ab, xb[i], acc[o][i]);
      }
    }
#pragma unroll
    for (int i = 0; i < Dm::ET; ++i)
      vq[i] += bdot4(kslice<S>(ta, R::GR2 + 16 * i), kslice<S>(ta, R::XH1 + 16 * i)) +
               bdot4(kslice<S>(tb, R::GR2 + 16 * i), kslice<S>(tb, R::XH1 + 16 * i));
  }
  T2O_DEV void finish(const DwGemmArgs& a, float* slab, int d) {
    if constexpr (Dm::MN) dw_tiles_store<Dm::HET, Dm::ET>(slab + a.G.M[d], E, acc);
    dw_vec_store<Dm::ET>(slab + a.G.g1[d], vq);
    // (the n1 slot is unused: t2o_unpack_grads derives d n1 from d c1, d c2)
    if (lane_g() == 0) {
#pragma unroll
      for (int i = 0; i < Dm::ET; ++i) slab[a.G.n1[d] + 16 * i + lane_c()] = 0.f;
    }
  }
};

template <int E, int H, int FF, int D, typename TT, int FMT>
struct DwRole<1, E, H, FF, D, TT, FMT> {
  using Dm = DwDims<E, H, FF, D, TT, 16, FMT>;
  using R = typename Dm::R;
  using Frag = typename std::conditional<Dm::BF, bf4, f4>::type;
  f4 acc[Dm::ET][Dm::HET];  // dN[gres feature][z feature]
  float vbu[Dm::ET];
  T2O_DEV void ready() {}
  T2O_DEV void init(const DwGemmArgs&, int, const TT*) {
#pragma unroll
    for (int o = 0; o < Dm::ET; ++o) {
      vbu[o] = 0.f;
#pragma unroll
      for (int i = 0; i < Dm::HET; ++i) acc[o][i] = zero4();
    }
  }
  T2O_DEV void tile(const TT* t) {
    constexpr int S = Dm::RSTR;
    Frag gb[Dm::ET];
#pragma unroll
    for (int o = 0; o < Dm::ET; ++o) {
      gb[o] = kslice<S>(t, R::GRES + 16 * o);
      vbu[o] += bsum4(gb[o]);
    }
    if constexpr (Dm::MN) {
#pragma unroll
      for (int i = 0; i < Dm::HET; ++i) {
        const Frag zb = kslice<S>(t, R::Z + 16 * i);
#pragma unroll
        for (int o = 0; o < Dm::ET; ++o) acc[o][i] = kmma(gb[o], zb, acc[o][i]);
      }
    }
  }
  T2O_DEV void tile2(const TT* ta, const TT* tb) {
    constexpr int S = Dm::RSTR;
    bf8 gb[Dm::ET];
#pragma unroll
    for (int o = 0; o < Dm::ET; ++o) {
      const bf4 a = kslice<S>(ta, R::GRES + 16 * o), b = kslice<S>(tb, R::GRES + 16 * o);
      gb[o] = cat8(a, b);
      vbu[o] += bsum4(a) + bsum4(b);
    }
    if constexpr (Dm::MN) {
#pragma unroll
      for (int i = 0; i < Dm::HET; ++i) {
        const bf8 zb = cat8(kslice<S>(ta, R::Z + 16 * i), kslice<S>(tb, R::Z + 16 * i));
#pragma unroll
        for (int o = 0; o < Dm::ET; ++o) acc[o][i] = kmma8(gb[o], zb, acc[o][i]);
      }
    }
  }
  T2O_DEV void finish(const DwGemmArgs& a, float* slab, int d) {
    if constexpr (Dm::MN) dw_tiles_store<Dm::ET, Dm::HET>(slab + a.G.N[d], H * E, acc);
    dw_vec_store<Dm::ET>(slab + a.G.bu[d], vbu);
  }
};

// FFN part PART of NPART: recompute y = x̂1 ⊙ g1 + n1, f1 = W1 y + c1 and gf1 =
// [f1 > 0] ⊙ W2ᵀ gr2 for the part's FH feature tiles as [records x features]
// MFMA tiles (lane (g, c) = records 4g..4g+3 of feature 16J + c — already the
// K-slice layout of the contraction), then dW2[e][J] += gr2 ⊗ relu(f1) and
// P[J][e] += gf1 ⊗ x̂1 (t2o_unpack_grads makes dW1 of P).
// Weight fragments: bf16 from the workgroup's LDS copy of the pack's
// (swizzled) bf16 image; fp32 straight from the pack (L2-resident).
// NPART 2: roles 2 / 3 of the full record (roles 0 / 1 contract dM, dN).
// NPART 4: the lean agent record (TapeRecA: dM / dN were accumulated by the
// BPTT) — all four waves of a block take an FFN quarter, with their weight
// fragments in registers for the launch, and the record's vector sums ride
// along (part 0: Q, part 1: d bu, part 2: d c2).  Round 4's split left two of
// the four waves with only those sums: the agent contraction ran 0.275 ms for
// 207 MB at the headline (0.75 TB/s, profiles/r4_h/prof/timeline.txt).
template <int PART, int NPART, int E, int H, int FF, int D, typename TT, int FMT>
struct DwFfn {
  using Dm = DwDims<E, H, FF, D, TT, 16, FMT>;
  using R = typename Dm::R;
  static constexpr int ET = Dm::ET, FH = Dm::FT / NPART;
  static constexpr bool WREG = NPART == 4 && Dm::BF;  // weight fragments held in registers
  static_assert(Dm::FT % NPART == 0, "FF must split into NPART parts of 16-feature tiles");
  using Frag = typename std::conditional<Dm::BF, bf4, f4>::type;
  f4 acc1[FH][ET];  // P rows of this part
  f4 acc2[ET][FH];  // dW2 columns of this part
  float vc1[FH], vc2[ET];
  float vq[ET], vbu[ET];  // NPART 4: Q (part 0), d bu (part 1)
  float c1v[FH];
  f4 g1r[ET], n1r[ET];  // fp32: LN1 affine of this lane's record-major features 16s + 4g .. +3
  Frag w1r[WREG ? FH : 1][ET], w2r[WREG ? FH : 1][ET];
  const TT* wl;     // bf16: LDS W1 [FF][E] then W2ᵀ [FF][E] of this block
  const float* wsrc;
  int64_t o1, o2;
  static constexpr bool DO_C2 = NPART == 2 ? PART == 0 : PART == 2;
  T2O_DEV void init(const DwGemmArgs& a, int d, const TT* wlds) {
    const int c = lane_c();
#pragma unroll
    for (int o = 0; o < FH; ++o) {
      vc1[o] = 0.f;
#pragma unroll
      for (int i = 0; i < ET; ++i) acc1[o][i] = acc2[i][o] = zero4();
    }
#pragma unroll
    for (int i = 0; i < ET; ++i) vc2[i] = vq[i] = vbu[i] = 0.f;
    wl = wlds + (size_t)d * 2 * FF * E;
    wsrc = a.pack;
    o1 = a.L.W1[d];
    o2 = a.L.W2T[d];
#pragma unroll
    for (int jt = 0; jt < FH; ++jt) c1v[jt] = a.pack[a.L.c1[d] + 16 * (PART * FH + jt) + c];
    if constexpr (Dm::BF) {  // the LDS W1 image carries g1; fold n1 into the bias
#pragma unroll
      for (int jt = 0; jt < FH; ++jt) {
        const float* w = a.pack + a.L.W1[d] + (int64_t)(16 * (PART * FH + jt) + c) * E;
        float acc = 0.f;
        for (int e = 0; e < E; ++e) acc = fmaf(w[e], a.pack[a.L.n1[d] + e], acc);
        c1v[jt] += acc;
      }
    } else {
#pragma unroll
      for (int s = 0; s < ET; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          g1r[s][r] = a.pack[a.L.g1[d] + 16 * s + 4 * lane_g() + r];
          n1r[s][r] = a.pack[a.L.n1[d] + 16 * s + 4 * lane_g() + r];
        }
    }
  }
  // after the first barrier (the LDS weight image is visible): the part's
  // fragments into registers
  T2O_DEV void ready() {
    if constexpr (WREG) {
#pragma unroll
      for (int jt = 0; jt < FH; ++jt)
#pragma unroll
        for (int s2 = 0; s2 < ET; ++s2) {
          w1r[jt][s2] = wfrag_lds(0, jt, s2);
          w2r[jt][s2] = wfrag_lds(1, jt, s2);
        }
    }
  }
  T2O_DEV Frag wfrag(int m, int jt, int s) const {
    if constexpr (WREG) return m ? w2r[jt][s] : w1r[jt][s];
    else return wfrag_lds(m, jt, s);
  }
  // fragment of W (0: W1, 1: W2ᵀ): row 16J + c, features 16s + 4g .. +3
  T2O_DEV Frag wfrag_lds(int m, int jt, int s) const {
    const int row = 16 * (PART * FH + jt) + lane_c();
    if constexpr (Dm::BF) {
      const TT* base = wl + (size_t)m * FF * E + (size_t)row * E;
      return ldb4(base + ((16 * s + 4 * lane_g()) ^ bf_swz(row, E)));
    } else {
      return ld4(wsrc + (m ? o2 : o1) + (int64_t)row * E + 16 * s + 4 * lane_g());
    }
  }
  // the recompute's record-major operand: bf16, x̂1 itself (g1 / n1 are folded
  // into the staged W1 and c1); fp32, y = x̂1 ⊙ g1 + n1 (the LN1 affine, layernorm_fwd)
  T2O_DEV Frag affine(Frag xh, int s) const {
    if constexpr (Dm::BF) {
      (void)s;
      return xh;
    } else {
      f4 y;
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = xh[r] * g1r[s][r] + n1r[s][r];
      return y;
    }
  }
  T2O_DEV void tile(const TT* t) {
    constexpr int S = Dm::RSTR;
    Frag yr[ET], gr[ET], xk[ET], gk[ET];
#pragma unroll
    for (int s = 0; s < ET; ++s) {
      yr[s] = affine(rslice<S>(t, R::XH1 + 16 * s), s);
      gr[s] = rslice<S>(t, R::GR2 + 16 * s);
      xk[s] = kslice<S>(t, R::XH1 + 16 * s);
      gk[s] = kslice<S>(t, R::GR2 + 16 * s);
      if (DO_C2) vc2[s] += bsum4(gk[s]);
      if (NPART == 4 && PART == 0) vq[s] += bdot4(gk[s], xk[s]);
      if (NPART == 4 && PART == 1) vbu[s] += bsum4(kslice<S>(t, R::GRES + 16 * s));
    }
#pragma unroll
    for (int jt = 0; jt < FH; ++jt) {
      f4 f1 = zero4(), gp = zero4();
#pragma unroll
      for (int s = 0; s < ET; ++s) {
        // [records x features]: A = record-major slice, B = weight rows
        f1 = kmma(yr[s], wfrag(0, jt, s), f1);
        gp = kmma(gr[s], wfrag(1, jt, s), gp);
      }
      f4 fr, gf;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = f1[r] + c1v[jt];
        fr[r] = fmaxf(v, 0.f);
        gf[r] = v > 0.f ? gp[r] : 0.f;
      }
      vc1[jt] += (gf[0] + gf[1]) + (gf[2] + gf[3]);
      Frag frb, gfb;
      if constexpr (Dm::BF) {
        frb = to_bf4(fr);
        gfb = to_bf4(gf);
      } else {
        frb = fr;
        gfb = gf;
      }
#pragma unroll
      for (int e = 0; e < ET; ++e) {
        acc2[e][jt] = kmma(gk[e], frb, acc2[e][jt]);  // dW2[e][J] += gr2 ⊗ relu(f1)
        acc1[jt][e] = kmma(gfb, xk[e], acc1[jt][e]);  // P[J][e] += gf1 ⊗ x̂1
      }
    }
  }
  // bf16, two tiles at once: the recompute contracts both feature tiles in one
  // 16x16x32 MFMA (K = 32 features), the weight-grad products both tiles' 32
  // records, and relu(f1) / gf1 of the two tiles convert 8-wide (packed)
  T2O_DEV void tile2(const TT* ta, const TT* tb) {
    static_assert(ET == 2, "the paired recompute contracts the two 16-feature tiles of E = 32");
    constexpr int S = Dm::RSTR;
    const TT* tt[2] = {ta, tb};
    bf8 yr[2], gr[2], xk[ET], gk[ET];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      yr[k] = cat8(rslice<S>(tt[k], R::XH1), rslice<S>(tt[k], R::XH1 + 16));
      gr[k] = cat8(rslice<S>(tt[k], R::GR2), rslice<S>(tt[k], R::GR2 + 16));
    }
#pragma unroll
    for (int s2 = 0; s2 < ET; ++s2) {
      const bf4 xa = kslice<S>(ta, R::XH1 + 16 * s2), xbb = kslice<S>(tb, R::XH1 + 16 * s2);
      const bf4 ga = kslice<S>(ta, R::GR2 + 16 * s2), gbb = kslice<S>(tb, R::GR2 + 16 * s2);
      xk[s2] = cat8(xa, xbb);
      gk[s2] = cat8(ga, gbb);
      if (DO_C2) vc2[s2] += bsum4(ga) + bsum4(gbb);
      if (NPART == 4 && PART == 0) vq[s2] += bdot4(ga, xa) + bdot4(gbb, xbb);
      if (NPART == 4 && PART == 1)
        vbu[s2] += bsum4(kslice<S>(ta, R::GRES + 16 * s2)) + bsum4(kslice<S>(tb, R::GRES + 16 * s2));
    }
#pragma unroll
    for (int jt = 0; jt < FH; ++jt) {
      const bf8 w1 = cat8(wfrag(0, jt, 0), wfrag(0, jt, 1)), w2 = cat8(wfrag(1, jt, 0), wfrag(1, jt, 1));
      f4 fr[2], gf[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const f4 f1 = kmma8(yr[k], w1, zero4()), gp = kmma8(gr[k], w2, zero4());
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = f1[r] + c1v[jt];
          fr[k][r] = fmaxf(v, 0.f);
          gf[k][r] = v > 0.f ? gp[r] : 0.f;
        }
        vc1[jt] += (gf[k][0] + gf[k][1]) + (gf[k][2] + gf[k][3]);
      }
      const bf8 frb = cvt8(fr[0], fr[1]), gfb = cvt8(gf[0], gf[1]);
#pragma unroll
      for (int e = 0; e < ET; ++e) {
        acc2[e][jt] = kmma8(gk[e], frb, acc2[e][jt]);  // dW2[e][J] += gr2 ⊗ relu(f1)
        acc1[jt][e] = kmma8(gfb, xk[e], acc1[jt][e]);  // P[J][e] += gf1 ⊗ x̂1
      }
    }
  }
  T2O_DEV void finish(const DwGemmArgs& a, float* slab, int d) {
    dw_tiles_store<FH, ET>(slab + a.G.W1[d] + (int64_t)16 * PART * FH * E, E, acc1);
    dw_tiles_store<ET, FH>(slab + a.G.W2[d] + 16 * PART * FH, FF, acc2);
    dw_vec_store<FH>(slab + a.G.c1[d] + 16 * PART * FH, vc1);
    if (DO_C2) dw_vec_store<ET>(slab + a.G.c2[d], vc2);
    if constexpr (NPART == 4 && PART == 0) {  // as role 0 of the full record
      dw_vec_store<ET>(slab + a.G.g1[d], vq);
      if (lane_g() == 0) {
#pragma unroll
        for (int i = 0; i < ET; ++i) slab[a.G.n1[d] + 16 * i + lane_c()] = 0.f;
      }
    }
    if constexpr (NPART == 4 && PART == 1) dw_vec_store<ET>(slab + a.G.bu[d], vbu);
  }
};
template <int E, int H, int FF, int D, typename TT, int FMT>
struct DwRole<2, E, H, FF, D, TT, FMT> : DwFfn<0, 2, E, H, FF, D, TT, FMT> {};
template <int E, int H, int FF, int D, typename TT, int FMT>
struct DwRole<3, E, H, FF, D, TT, FMT> : DwFfn<1, 2, E, H, FF, D, TT, FMT> {};
// the lean agent record: four FFN quarters (roles 4 + q)
template <int E, int H, int FF, int D, typename TT, int FMT>
struct DwRole<4, E, H, FF, D, TT, FMT> : DwFfn<0, 4, E, H, FF, D, TT, FMT> {};
template <int E, int H, int FF, int D, typename TT, int FMT>
struct DwRole<5, E, H, FF, D, TT, FMT> : DwFfn<1, 4, E, H, FF, D, TT, FMT> {};
template <int E, int H, int FF, int D, typename TT, int FMT>
struct DwRole<6, E, H, FF, D, TT, FMT> : DwFfn<2, 4, E, H, FF, D, TT, FMT> {};
template <int E, int H, int FF, int D, typename TT, int FMT>
struct DwRole<7, E, H, FF, D, TT, FMT> : DwFfn<3, 4, E, H, FF, D, TT, FMT> {};

// One wave's whole launch for its role (every role runs the same pipeline and
// the same barrier sequence; the roles only differ in what they read).
// Pipeline: LDS double buffer, register ring of two, prefetch distance 2.
template <int ROLE, int E, int H, int FF, int D, typename TT, int RT, int FMT>
T2O_DEV void dw_run(const DwGemmArgs& a, int wg, int nwg, TT* buf0, TT* buf1, const TT* wlds, int d) {
  using Dm = DwDims<E, H, FF, D, TT, RT, FMT>;
  const int64_t ngroups = (a.ntiles + Dm::TG - 1) / Dm::TG;
  const int64_t nj = (int64_t)wg < ngroups ? (ngroups - 1 - wg) / nwg + 1 : 0;
  DwRole<ROLE, E, H, FF, D, TT, FMT> st;
  st.init(a, d, wlds);
  auto compute = [&](const TT* buf) {
    if constexpr (Dm::BF && Dm::TG % 2 == 0 && E == 32 && FMT == 1) {
#pragma unroll
      for (int tt = 0; tt < Dm::TG; tt += 2) {
        st.tile2(buf + (d * Dm::TG + tt) * Dm::TSTR, buf + (d * Dm::TG + tt + 1) * Dm::TSTR);
        T2O_FENCE();
      }
    } else {
#pragma unroll
      for (int tt = 0; tt < Dm::TG; ++tt) {
        st.tile(buf + (d * Dm::TG + tt) * Dm::TSTR);
        T2O_FENCE();  // keep the next tile's LDS reads from being hoisted over these MFMAs
      }
    }
  };
  u4v r0[Dm::NLD], r1[Dm::NLD];
  if (nj > 0) dw_load<Dm, TT>(a, wg, nwg, 0, r0);
  if (nj > 1) dw_load<Dm, TT>(a, wg, nwg, 1, r1);
  if (nj > 0) dw_store<Dm, TT>(buf0, r0);
  if (nj > 1) dw_store<Dm, TT>(buf1, r1);
  if (nj > 2) dw_load<Dm, TT>(a, wg, nwg, 2, r0);
  if (nj > 3) dw_load<Dm, TT>(a, wg, nwg, 3, r1);
  __syncthreads();
  st.ready();
  for (int64_t j = 0; j < nj; j += 2) {
    compute(buf0);
    __syncthreads();
    if (j + 2 < nj) dw_store<Dm, TT>(buf0, r0);
    if (j + 4 < nj) dw_load<Dm, TT>(a, wg, nwg, j + 4, r0);
    if (j + 1 >= nj) break;
    compute(buf1);
    __syncthreads();
    if (j + 3 < nj) dw_store<Dm, TT>(buf1, r1);
    if (j + 5 < nj) dw_load<Dm, TT>(a, wg, nwg, j + 5, r1);
  }
  st.finish(a, a.slabs + (size_t)wg * a.slab_stride, d);
}

// LDS elements (of TT) one workgroup of a contraction instance takes
template <int E, int H, int FF, int D, typename TT, int FMT>
constexpr size_t dw_lds_elems() {
  using Dm = DwDims<E, H, FF, D, TT, 16, FMT>;
  return (size_t)2 * Dm::GELEM + (Dm::BF ? (size_t)D * 2 * FF * E : 0);
}

// One workgroup's contraction: workgroup wg of nwg over the tape of `a`.
template <int E, int H, int FF, int D, typename TT, int RT, int FMT>
T2O_DEV void dw_gemm_wg(const DwGemmArgs& a, int wg, int nwg, float* smem) {
  using Dm = DwDims<E, H, FF, D, TT, RT, FMT>;
  TT* const buf0 = reinterpret_cast<TT*>(smem);
  TT* const buf1 = buf0 + Dm::GELEM;
  TT* const wlds = buf1 + Dm::GELEM;  // bf16: [D][W1, W2ᵀ][FF][E] (the pack's swizzled image)
  if constexpr (Dm::BF) {  // made visible by dw_run's first barrier
    // W2ᵀ: the pack's swizzled bf16 image; W1: folded with the LN1 gain,
    // W1[J][e]·g1[e], rounded to bf16 in the same swizzled placement, so the
    // recompute f1 = (W1 ⊙ g1) x̂1 + (c1 + W1 n1) reads the tape's x̂1 directly
    const TT* img = reinterpret_cast<const TT*>(a.pack + a.L.total);
    constexpr int MAT = FF * E;
    for (int q = threadIdx.x; q < D * 2 * MAT / Dm::PER; q += Dm::NT) {
      const int e = q * Dm::PER, dd = e / (2 * MAT), m = (e / MAT) & 1, k = e % MAT;
      if (m) {
        *reinterpret_cast<u4v*>(wlds + e) = *reinterpret_cast<const u4v*>(img + a.L.W2T[dd] + k);
      } else {
        const int row = k / E, c0 = (k % E) ^ bf_swz(row, E);  // 8 consecutive image slots = 8 columns
        const float* w = a.pack + a.L.W1[dd] + (int64_t)row * E + c0;
        const float* g = a.pack + a.L.g1[dd] + c0;
#pragma unroll
        for (int i = 0; i < Dm::PER; ++i) wlds[e + i] = (TT)(w[i] * g[i]);
      }
    }
  }
  if constexpr (RT < 16) {  // compact tiles: LDS records RT..15 stay zero (they add nothing)
    for (int q = threadIdx.x; q < 2 * D * Dm::TG * (16 - RT) * Dm::CPR; q += Dm::NT) {
      const int cr = q % Dm::CPR, rr = q / Dm::CPR;
      const int rec = RT + rr % (16 - RT), tix = rr / (16 - RT);  // tix over both buffers
      *reinterpret_cast<u4v*>(buf0 + tix * Dm::TSTR + rec * Dm::RSTR + cr * Dm::PER) = u4v{0u, 0u, 0u, 0u};
    }
  }
  const int w = wave_id();
  // Waves w and w + 4 share a SIMD.  Roles 2/3 (FFN halves: 32 MFMAs per tile
  // plus the W1/W2ᵀ reads) weigh about 2.7x roles 0/1 (12 MFMAs), so block 1
  // rotates its roles by two: every SIMD holds one light and one heavy role.
  const int d = w >> 2, role = (w + 2 * d) & 3;
  if constexpr (FMT == 1) {  // lean agent record: four equal FFN quarters
    switch (w & 3) {
      case 0: dw_run<4, E, H, FF, D, TT, RT, FMT>(a, wg, nwg, buf0, buf1, wlds, d); break;
      case 1: dw_run<5, E, H, FF, D, TT, RT, FMT>(a, wg, nwg, buf0, buf1, wlds, d); break;
      case 2: dw_run<6, E, H, FF, D, TT, RT, FMT>(a, wg, nwg, buf0, buf1, wlds, d); break;
      default: dw_run<7, E, H, FF, D, TT, RT, FMT>(a, wg, nwg, buf0, buf1, wlds, d); break;
    }
  } else {
    // the heavy (FFN-half) wave issues first on its SIMD, the light one fills its
    // gaps (A/B: mixer_dw 0.256 -> 0.249 ms; prioritising the light roles: no gain)
    if (role >= 2) __builtin_amdgcn_s_setprio(1);
    switch (role) {  // wave-uniform; the four paths issue the same barriers
      case 0: dw_run<0, E, H, FF, D, TT, RT, FMT>(a, wg, nwg, buf0, buf1, wlds, d); break;
      case 1: dw_run<1, E, H, FF, D, TT, RT, FMT>(a, wg, nwg, buf0, buf1, wlds, d); break;
      case 2: dw_run<2, E, H, FF, D, TT, RT, FMT>(a, wg, nwg, buf0, buf1, wlds, d); break;
      default: dw_run<3, E, H, FF, D, TT, RT, FMT>(a, wg, nwg, buf0, buf1, wlds, d); break;
    }
  }
}

template <int E, int H, int FF, int D, int KIND, typename TT, int RT, int FMT>
__global__ __launch_bounds__(256 * D) void dw_gemm_kernel(DwGemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  dw_gemm_wg<E, H, FF, D, TT, RT, FMT>(a, blockIdx.x, gridDim.x, smem);
}

// Both backwards' tapes in ONE grid (t2o_bwd_tape_contract with two tapes): workgroups
// [0, n0) contract tape 0 (record format 0: the mixer's), the rest tape 1
// (format FMT1: the agent's).  After the agent BPTT the two contractions are the
// update's tail; as one launch their workgroups share the chip from the first
// wave on and the second launch's ramp and gap disappear.
template <int E, int H, int FF, int D, typename TT, int FMT1>
__global__ __launch_bounds__(256 * D) void dw_gemm_pair_kernel(DwGemmArgs a0, DwGemmArgs a1, int n0) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  if ((int)blockIdx.x < n0) {
    dw_gemm_wg<E, H, FF, D, TT, 16, 0>(a0, blockIdx.x, n0, smem);
  } else {
    dw_gemm_wg<E, H, FF, D, TT, 16, FMT1>(a1, blockIdx.x - n0, gridDim.x - n0, smem);
  }
}

template <int E, int H, int FF, int D, typename TT, int FMT>
int launch_dw_gemm(int kind, const void* tape, int64_t ntiles, const float* pack, float* slabs, const t2o_layout& L,
                   const t2o_layout& G, int nslab, hipStream_t stream) {
  using Dm = DwDims<E, H, FF, D, TT, 16, FMT>;
  if (nslab < 1) return T2O_EINVAL;
  DwGemmArgs a{};
  a.tape = tape;
  a.ntiles = ntiles;
  a.slabs = slabs;
  a.slab_stride = G.grad_total;
  a.pack = pack;
  a.L = L;
  a.G = G;
  (void)sizeof(Dm);
  const size_t lds = sizeof(TT) * dw_lds_elems<E, H, FF, D, TT, FMT>();
  // (every tuned mixer writes its records as one compact stream of 16-record tiles)
  auto kern = kind == 0 ? dw_gemm_kernel<E, H, FF, D, 0, TT, 16, FMT> : dw_gemm_kernel<E, H, FF, D, 1, TT, 16, 0>;
  if (lds > 160 * 1024) return T2O_EUNSUPPORTED;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(nslab), dim3(256 * D), lds, stream, a);
  return (int)hipGetLastError();
}

static DwGemmArgs dw_args(const void* tape, int64_t ntiles, const float* pack, float* slabs, const t2o_layout& L) {
  DwGemmArgs a{};
  a.tape = tape;
  a.ntiles = ntiles;
  a.slabs = slabs;
  a.pack = pack;
  a.L = L;
  grad_layout(L, a.G);
  a.slab_stride = a.G.grad_total;
  return a;
}

template <int E, int H, int FF, int D, typename TT, int FMT1>
int launch_dw_gemm_pair(const DwGemmArgs& a0, int n0, const DwGemmArgs& a1, int n1, hipStream_t stream) {
  constexpr size_t l0 = dw_lds_elems<E, H, FF, D, TT, 0>(), l1 = dw_lds_elems<E, H, FF, D, TT, FMT1>();
  const size_t lds = sizeof(TT) * (l0 > l1 ? l0 : l1);
  if (lds > 160 * 1024) return T2O_EUNSUPPORTED;
  auto kern = dw_gemm_pair_kernel<E, H, FF, D, TT, FMT1>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(n0 + n1), dim3(256 * D), lds, stream, a0, a1, n0);
  return (int)hipGetLastError();
}

}  // namespace t2o

using namespace t2o;

extern "C" int64_t t2o_bwd_tape_floats(const t2o_layout* L, int64_t tiles) {
  if (!L || tiles < 0) return -1;
  if (L->generic) return gen_tape_floats(L, tiles);
  const int64_t elems = (int64_t)L->D * tiles * tape_tile_records(*L) * (4 * L->E + 2 * L->H * L->E);
  return L->prec ? (elems + 1) / 2 : elems;
}

extern "C" int64_t t2o_bwd_tape_tiles(const t2o_layout* L, int B, int T, int A) {
  if (!L || B < 1 || T < 1 || A < 1) return -1;
  if (L->kind == 0) return (int64_t)T * (((int64_t)B * A + 15) / 16);
  if (A != L->n_agents) return -1;
  const int64_t Q = A + 3;  // the mixer's query rows: A weight rows + 3 hyper tokens
  // tuned mixers write each block's records as one compact stream, (step,
  // episode, query row) in order, cut into 16-record tiles (t2o_mixer.hip); a
  // generic mixer, one tile-set per (episode, step)
  if (!L->generic) return ((int64_t)B * T * Q + 15) / 16;
  return (int64_t)B * T * ((Q + 15) / 16);
}

static int contract_one(const t2o_layout* L, const float* pack, const void* tape, int64_t tiles,
                                        float* gslabs, int nslab, int rec_format, void* stream) {
  if (!L || !pack || !tape || !gslabs || tiles < 0 || nslab < 1 || rec_format < 0 || rec_format > 1 ||
      (rec_format == 1 && (L->kind != 0 || !L->prec || L->generic)))
    return T2O_EINVAL;
  if (L->generic) return gen_tape_contract(L, tape, tiles, gslabs, nslab, (hipStream_t)stream);
  t2o_layout G;
  grad_layout(*L, G);
  int rc = T2O_EUNSUPPORTED;
  if (rec_format == 1) {
    T2O_DISPATCH_NET(L->E, L->H, L->D, L->FF,
                 rc = (launch_dw_gemm<E_, H_, FF_, D_, __bf16, 1>(0, tape, tiles, pack, gslabs, *L, G, nslab,
                                                                      (hipStream_t)stream)));
    return rc;
  }
  T2O_DISPATCH_NET(L->E, L->H, L->D, L->FF,
               rc = (L->prec ? launch_dw_gemm<E_, H_, FF_, D_, __bf16, 0>(L->kind, tape, tiles, pack, gslabs, *L,
                                                                          G, nslab, (hipStream_t)stream)
                             : launch_dw_gemm<E_, H_, FF_, D_, float, 0>(L->kind, tape, tiles, pack, gslabs, *L, G,
                                                                         nslab, (hipStream_t)stream)));
  return rc;
}

static int contract_pair(const t2o_layout* Lm, const float* pack_m, const void* tape_m,
                                          int64_t tiles_m, float* slabs_m, int nslab_m, const t2o_layout* La,
                                          const float* pack_a, const void* tape_a, int64_t tiles_a,
                                          float* slabs_a, int nslab_a, int rec_format_a, void* stream) {
  if (!Lm || !La || Lm->kind != 1 || La->kind != 0) return T2O_EINVAL;
  if (!pack_m || !tape_m || !slabs_m || tiles_m < 0 || nslab_m < 1 || !pack_a || !tape_a || !slabs_a ||
      tiles_a < 0 || nslab_a < 1 || rec_format_a < 0 || rec_format_a > 1 || (rec_format_a == 1 && !La->prec))
    return T2O_EINVAL;
  // one grid needs one kernel instance: both networks tuned, same (E, H, D, FF) and precision
  const bool same = !Lm->generic && !La->generic && Lm->E == La->E && Lm->H == La->H && Lm->D == La->D &&
                    Lm->FF == La->FF && Lm->prec == La->prec;
  hipStream_t s = (hipStream_t)stream;
  if (!same) {
    int rc = contract_one(Lm, pack_m, tape_m, tiles_m, slabs_m, nslab_m, 0, stream);
    return rc ? rc : contract_one(La, pack_a, tape_a, tiles_a, slabs_a, nslab_a, rec_format_a, stream);
  }
  const DwGemmArgs am = dw_args(tape_m, tiles_m, pack_m, slabs_m, *Lm);
  const DwGemmArgs aa = dw_args(tape_a, tiles_a, pack_a, slabs_a, *La);
  int rc = T2O_EUNSUPPORTED;
  T2O_DISPATCH_NET(La->E, La->H, La->D, La->FF,
                   rc = (La->prec ? (rec_format_a == 1
                                         ? launch_dw_gemm_pair<E_, H_, FF_, D_, __bf16, 1>(am, nslab_m, aa, nslab_a, s)
                                         : launch_dw_gemm_pair<E_, H_, FF_, D_, __bf16, 0>(am, nslab_m, aa, nslab_a, s))
                                  : launch_dw_gemm_pair<E_, H_, FF_, D_, float, 0>(am, nslab_m, aa, nslab_a, s)));
  return rc;
}

extern "C" int t2o_bwd_tape_contract(const t2o_tape_args* first, const t2o_tape_args* second, void* stream) {
  if (!first) return T2O_EINVAL;
  if (!second)
    return contract_one(first->L, first->pack, first->tape, first->tiles, first->gslabs, first->nslab,
                        first->rec_format, stream);
  if (first->rec_format != 0) return T2O_EINVAL;  // (the first of a pair is the mixer's tape)
  return contract_pair(first->L, first->pack, first->tape, first->tiles, first->gslabs, first->nslab, second->L,
                       second->pack, second->tape, second->tiles, second->gslabs, second->nslab, second->rec_format,
                       stream);
}
