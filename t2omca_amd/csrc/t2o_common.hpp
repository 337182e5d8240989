// t2o_common.hpp — CDNA4 (gfx950) building blocks shared by the T2OMCA kernels.
//
// Register layout ("T-layout").  A wave owns a tile of 16 ROWS (agent: one
// (episode, agent) sequence per row; mixer: one query token per row).  Lane
// l = 16*g + c holds row c; its lane group g (0..3) holds features
// 16*t + 4*g + r (r = 0..3) of every 16-feature tile t, i.e. an activation
// vector of 16*T features is `f4 v[T]`.  This is exactly the D layout of
// v_mfma_f32_16x16x4_f32 when the MFMA computes   y^T = W · x^T
// (out-features on the MFMA M axis, rows on the N axis), and — because the
// contraction order is free — the same registers are directly the B operand
// of the next MFMA: step s of a 16-wide K tile feeds register r = s, so a
// chain of projections never moves activations between lanes or through LDS.
// Weights are the A operand: lane (g, c) of step s needs W[16o+c][16i+4g+s],
// i.e. ONE 16-byte load of 4 consecutive in-features of a row-major W.
//
// All arithmetic here is fp32; v_mfma_f32_16x16x4_f32 is an exact fp32 FMA
// chain (MI355X_MICROARCH.md §Matrix cores), so results track the reference's
// fp32 CPU path to rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/t2omca.h"

typedef float f4 __attribute__((ext_vector_type(4)));

#define T2O_DEV __device__ __forceinline__

// Stream keys of the counter-based uniforms (env_spec.uniforms): XOR-ed into the
// seed of every stream but the env's, so the env, the ε-greedy selector and the
// PER sampler draw independent sequences from one user seed.
#define T2O_STREAM_MAC 0x4D41435354524D31ull  // "MACSTRM1"
#define T2O_STREAM_PER 0x5045525354524D31ull  // "PERSTRM1"

namespace t2o {

T2O_DEV int lane_c() { return threadIdx.x & 15; }
T2O_DEV int lane_g() { return (threadIdx.x >> 4) & 3; }
T2O_DEV int wave_id() { return threadIdx.x >> 6; }

T2O_DEV f4 zero4() { return f4{0.f, 0.f, 0.f, 0.f}; }

// Scheduling fence: stops the machine scheduler from hoisting the (activation-
// independent) weight loads of later stages above the current one, which
// otherwise keeps every layer's weight fragments live at once and spills.
#define T2O_FENCE() __builtin_amdgcn_sched_barrier(0)

// Diagnostic builds only (-DT2O_PHASE_PROF): cycle stamps of one workgroup's waves
#ifdef T2O_PHASE_PROF
__device__ long long t2o_mark_buf[8][8];
__device__ long long t2o_prof_buf[128 * 8 * 4];  // [slot][wave][delta]
#define T2O_MARK(n)                                                                         \
  do {                                                                                     \
    if (blockIdx.x == 7 && (threadIdx.x & 63) == 0) t2o_mark_buf[threadIdx.x >> 6][n] = clock64(); \
  } while (0)
// deltas between marks 0..NM of this wave into slot `slot` (WG 7, first 8 waves)
#define T2O_PROF_SAVE(slot, NM)                                                                   \
  do {                                                                                           \
    const int w_ = threadIdx.x >> 6;                                                             \
    if (blockIdx.x == 7 && (threadIdx.x & 63) == 0 && (slot) < 128 && w_ < 8)                     \
      for (int m_ = 0; m_ < (NM) && m_ < 4; ++m_)                                               \
        t2o_prof_buf[((slot) * 8 + w_) * 4 + m_] = t2o_mark_buf[w_][m_ + 1] - t2o_mark_buf[w_][m_]; \
  } while (0)
// absolute stamp into slot/idx (timeline builds: -DT2O_PHASE_PROF -DT2O_TIMELINE)
#define T2O_STAMP(slot, idx)                                                                     \
  do {                                                                                           \
    const int w_ = threadIdx.x >> 6;                                                             \
    if (blockIdx.x == 7 && (threadIdx.x & 63) == 0 && (slot) < 128 && w_ < 8)                     \
      t2o_prof_buf[((slot) * 8 + w_) * 4 + (idx)] = clock64();                                   \
  } while (0)
#define T2O_PROF_READER(fn)                                                          \
  extern "C" int fn(long long* host_out) {                                          \
    return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(t2o_prof_buf), sizeof(t2o_prof_buf)); \
  }
#else
#define T2O_MARK(n) \
  do {            \
  } while (0)
#define T2O_PROF_SAVE(slot, NM) \
  do {                        \
  } while (0)
#define T2O_PROF_READER(fn)
#define T2O_STAMP(slot, idx) \
  do {                     \
  } while (0)
#endif

// Intra-wave LDS hand-off (one wave's lanes exchange rows through LDS): the
// hardware keeps a wave's LDS operations in order, but __builtin_amdgcn_wave_barrier
// alone is no memory barrier to the COMPILER, which may move a load of another
// lane's row above this lane's store wherever it can prove the two addresses differ
// for one lane.  The wavefront-scope fences make the hand-off an ordering point for
// the optimiser; they emit no instructions.  (The bare barrier in the mixer kernels
// let an edit elsewhere reorder such a pair: DESIGN §9.)
T2O_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Debug builds only (tools/build_debug.sh, -DT2O_DEBUG_POISON=1): every kernel
// first fills its launch's whole dynamic LDS allocation with 0xFFFFFFFF (a NaN
// in fp32 and in both bf16 halves), so a read of LDS no code of the launch wrote
// turns into a NaN in the results instead of whatever the previous workgroup on
// that CU left there.  The group segment size comes from the dispatch packet
// (hsa_kernel_dispatch_packet_t.group_segment_size, byte offset 28).
#ifndef T2O_DEBUG_POISON
#define T2O_DEBUG_POISON 0
#endif
#if T2O_DEBUG_POISON && defined(__HIP_DEVICE_COMPILE__)
#define T2O_LDS_POISON(smem)                                                                          \
  do {                                                                                               \
    const uint32_t seg_ = reinterpret_cast<const uint32_t*>(__builtin_amdgcn_dispatch_ptr())[7];     \
    const uint32_t n_ = (seg_ - __builtin_amdgcn_groupstaticsize()) / 4;                             \
    const uint32_t nthr_ = blockDim.x * blockDim.y * blockDim.z;                                     \
    for (uint32_t i_ = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z); i_ < n_; i_ += nthr_) reinterpret_cast<uint32_t*>(smem)[i_] = ~0u; \
    __syncthreads();                                                                                 \
  } while (0)
#else
#define T2O_LDS_POISON(smem) \
  do {                      \
  } while (0)
#endif

T2O_DEV f4 mfma4(float a, float b, f4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
}

T2O_DEV f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

typedef float f2 __attribute__((ext_vector_type(2)));
// a·b over 4 features as (a0 b0 + a2 b2) + (a1 b1 + a3 b3): one v_pk_mul_f32, one
// v_pk_fma_f32 and an add (the lane's partial of an entity score)
T2O_DEV float dot4_pk(f4 a, f4 b) {
  const f2 t = __builtin_elementwise_fma(a.zw, b.zw, a.xy * b.xy);
  return t.x + t.y;
}

// e^x for softmax arguments (x <= 0, -inf allowed): one v_exp_f32 (2^y, ~1 ulp)
// of y = x·log2(e) instead of libm expf's range-reduced ~10-instruction expansion.
// Relative error ≈ |x|·2^-24 + 1 ulp, far inside the fp32 parity bar.
T2O_DEV float exp_fast(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
// 1/x and 1/sqrt(x) as single v_rcp_f32 / v_rsq_f32 (~1 ulp) instead of the
// IEEE division / sqrt expansions (softmax normaliser, LayerNorm).
T2O_DEV float rcp_fast(float x) { return __builtin_amdgcn_rcpf(x); }
T2O_DEV float rsqrt_fast(float x) { return __builtin_amdgcn_rsqf(x); }
// p[i] when ok, else 0 — one unconditional load from a clamped index (no branch
// around the load; the index must be valid when ok, and 0 is always valid).
T2O_DEV float ld_or0(const float* __restrict__ p, int64_t i, bool ok) {
  const float v = p[ok ? i : 0];
  return ok ? v : 0.f;
}
T2O_DEV void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// acc += W[16o.. , 16i..] (16x16 tile of row-major W, leading dim ldw) · x_tile
T2O_DEV f4 mma_tile(const float* __restrict__ W, int ldw, int o, int i, f4 x, f4 acc, bool = true) {
  const f4 w = ld4(W + (size_t)(16 * o + lane_c()) * ldw + 16 * i + 4 * lane_g());
  acc = mfma4(w[0], x[0], acc);
  acc = mfma4(w[1], x[1], acc);
  acc = mfma4(w[2], x[2], acc);
  acc = mfma4(w[3], x[3], acc);
  return acc;
}

// y[0..OT) = W[16*OT x 16*IT] · x[0..IT)  (T-layout in, T-layout out)
// (HOIST: see the bf16 overload; nothing to hoist in fp32)
// ACC: accumulate onto y (the caller's bias / residual) instead of zero
template <int OT, int IT, bool HOIST = true, bool ACC = false>
T2O_DEV void matvec(const float* __restrict__ W, int ldw, const f4* x, f4* y, bool = true) {
#pragma unroll
  for (int o = 0; o < OT; ++o) {
    f4 acc = ACC ? y[o] : zero4();
#pragma unroll
    for (int i = 0; i < IT; ++i) acc = mma_tile(W, ldw, o, i, x[i], acc);
    y[o] = acc;
  }
}

// y[0..OT) = Wᵀ · x[0..IT)  for row-major W [16*IT rows][ldw >= 16*OT] — the
// transposed product read straight from the same (LDS-resident) copy: lane
// (g, c) of step s needs Wᵀ[16o+c][16i+4g+s] = W[16i+4g+s][16o+c], one scalar
// read per MFMA step (consecutive c -> consecutive banks).
template <int OT, int IT>
T2O_DEV void matvec_t(const float* __restrict__ W, int ldw, const f4* x, f4* y) {
  const int c = lane_c(), g = lane_g();
#pragma unroll
  for (int o = 0; o < OT; ++o) {
    f4 acc = zero4();
#pragma unroll
    for (int i = 0; i < IT; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma4(W[(16 * i + 4 * g + s) * ldw + 16 * o + c], x[i][s], acc);
    y[o] = acc;
  }
}

// ---- bf16 MFMA operands (prec 1) ---------------------------------------------
// v_mfma_f32_16x16x16_bf16 takes, per lane, 4 consecutive K values of A and B:
// lane (g, c) gives A[c][4g..4g+3] and B[4g..4g+3][c] — exactly one T-layout
// f4 rounded to bf16 for B and 4 consecutive bf16 of a weight row for A, so a
// 16x16 tile is ONE MFMA instead of four f32 ones.  16x16x32 takes 8 K values
// per lane; feeding it (tile i, tile i+1) pairs with the same pairing in A and
// B contracts two 16-feature tiles per instruction.  Accumulation is fp32.
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));

// f32 -> bf16 (round to nearest even).  hipcc (ROCm 7.2, gfx950) emits the
// packed v_cvt_pk_bf16_f32 only for an 8-wide conversion; a lone f4 is
// scalarised (four conversions with a dummy second source + two v_perm_b32: six
// VALU for two).  Convert f4 PAIRS through cvt8 wherever two tiles are
// converted together (to_bf4_pairs, the 16x16x32 operands of matvec / KeyFrags).
T2O_DEV bf4 to_bf4(f4 x) { return __builtin_convertvector(x, bf4); }
T2O_DEV bf8 cvt8(f4 a, f4 b) { return __builtin_convertvector(__builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7), bf8); }
T2O_DEV bf4 lo4(bf8 v) { return __builtin_shufflevector(v, v, 0, 1, 2, 3); }
T2O_DEV bf4 hi4(bf8 v) { return __builtin_shufflevector(v, v, 4, 5, 6, 7); }
T2O_DEV bf4 ldb4(const __bf16* p) { return *reinterpret_cast<const bf4*>(p); }
// ReLU of bf16 operands on their bit patterns: a bf16 is negative (or -0) iff
// its sign bit is set, i.e. iff it is negative as an int16, so max_i16(x, 0) is
// relu(x) — packed v_pk_max_i16, bit-identical to rounding relu(x) in fp32
// (both give +0 for every x <= 0).
typedef short s8v __attribute__((ext_vector_type(8)));
T2O_DEV bf8 relu_bf8(bf8 x) {
  const s8v v = __builtin_bit_cast(s8v, x);
  return __builtin_bit_cast(bf8, __builtin_elementwise_max(v, s8v{0, 0, 0, 0, 0, 0, 0, 0}));
}
// A weight fragment (4 bf16 of one image row).  From LDS it is a volatile
// ds_read_b64: the compiler then loads each half of a 16x16x32 operand straight
// into its registers instead of fusing the fragments of two rows into one
// ds_read2st64_b64 (8 LDS cycles, banked mod 32 — the image swizzle is laid out
// for ds_read_b64's mod-64 banks) and assembling the operand with four v_mov.
// Per step loop: mixer_fwd 2217 -> 2103 instructions, mixer BPTT block-1 wave
// 2619 -> 2497, block-0 2033 -> 1926, agent_fwd 2403 -> 2298 (gfx950 ISA).  The
// address-space test folds at compile time (the weights' pointer comes from
// stage_weights or global_weights).
T2O_DEV bf4 ldw4(const __bf16* p) {
  typedef __attribute__((address_space(3))) const volatile bf4 lds_bf4;
  if (__builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)p)) return *(lds_bf4*)(p);
  return *reinterpret_cast<const bf4*>(p);
}
T2O_DEV f4 mfma_b16(bf4 a, bf4 b, f4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s4v, a), __builtin_bit_cast(s4v, b), acc, 0, 0,
                                                    0);
}
T2O_DEV f4 mfma_b32(bf4 a0, bf4 a1, bf4 b0, bf4 b1, f4 acc) {
  const bf8 a = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
  const bf8 b = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}

#ifndef T2O_SWZ_HOIST  // see matvec (bf16)
#define T2O_SWZ_HOIST 1
#endif

// Bank-conflict-free bf16 weight rows.  The bf16 image stores element
// (r, col) at r*ld + (col ^ bf_swz(r, ld)) — an XOR of whole 8-element groups,
// so the 4 (or 8) consecutive K values a lane loads stay contiguous — and the
// readers apply the same XOR.  Only the row's lane index matters:
// bf_swz(16o + c, ld) == bf_swz(c, ld).  The group index x(r) (sw = 8·x) is
// chosen per row length so that BOTH read kinds are conflict-free
// (MI355X_MICROARCH.md §LDS: ds_read_b64 and ds_read_b64_tr_b16 bank = dword
// address mod 64, lanes 0-31 and 32-63 separately):
//  * matvec (ds_read_b64): lane (g, c) reads 2 dwords of row c at group
//    (2i + g/2) ^ x(c): x must be a bijection over the rows that share a bank
//    base (row r starts at dword r·ld/2 mod 64);
//  * matvec_tr (ds_read_b64_tr_b16): lane (g, c) reads 8 B of row
//    q = 4g + (c >> 2) in output tile o, i.e. one 8-dword window per row, at
//    window (o ^ (x >> 1)) of the row: x >> 1 must separate the rows q of a
//    32-lane half that share a bank base.
//  ld ≡ 0 mod 128 (one bank base, 16 groups): x = (r & 7) << 1 | r >> 3 & 1
//  ld ≡ 64 mod 128 (two bases, 8 groups):     x = (r >> 1 & 3) << 1 | r >> 3 & 1
//  ld ≡ 32 mod 64  (four bases, 4 groups):    x = (r >> 2 & 1) << 1 | r >> 3 & 1
//  ld = 16         (eight bases, 2 groups):   x = r >> 3 & 1
// (Round 2 used x = r >> 2 & 3 for every ld ≡ 0 mod 32: fine for ld = 32 / 96
// matvec reads, but 4-way conflicted at ld = 128 (the FFN's W2 and W1ᵀ) and
// 2-way / 8-way on the transposed reads at ld = 32 / 128.)
__host__ __device__ inline int bf_swz(int row, int ld) {
  if (ld % 128 == 0) return 8 * (((row & 7) << 1) | ((row >> 3) & 1));
  if (ld % 64 == 0) return 8 * ((((row >> 1) & 3) << 1) | ((row >> 3) & 1));
  if (ld % 32 == 0) return 8 * ((((row >> 2) & 1) << 1) | ((row >> 3) & 1));
  return 8 * ((row >> 3) & 1);
}

T2O_DEV f4 mma_tile(const __bf16* __restrict__ W, int ldw, int o, int i, f4 x, f4 acc, bool vol = true) {
  const int c = lane_c();
  const __bf16* p = W + (size_t)(16 * o + c) * ldw + ((16 * i + 4 * lane_g()) ^ bf_swz(c, ldw));
  return mfma_b16(vol ? ldw4(p) : ldb4(p), to_bf4(x), acc);
}

// acc + A·B for a lone 16-wide K tail.  AFTER_B32: acc is a v_mfma_f32_16x16x32_bf16
// result — chained in place, the 16x16x16 would read it stale (hipcc 7.2 issues the
// pair with 0-4 wait states; t2o_probe_xdl_hazards), so the tail is
// accumulated on its own and added by VALU (which hipcc pads correctly).
template <bool AFTER_B32>
T2O_DEV f4 chain_tail_b16(bf4 a, bf4 b, f4 acc) {
  if constexpr (AFTER_B32) return acc + mfma_b16(a, b, zero4());
  else return mfma_b16(a, b, acc);
}

// y[0..OT) = W · x[0..IT), bf16 weights and operands, fp32 accumulate
template <int OT, int IT, bool HOIST = T2O_SWZ_HOIST, bool ACC = false>
T2O_DEV void matvec_b(const __bf16* __restrict__ W, int ldw, const bf4* xb, f4* y, bool vol = true);
template <int OT, int IT, bool HOIST = T2O_SWZ_HOIST, bool ACC = false>
T2O_DEV void matvec(const __bf16* __restrict__ W, int ldw, const f4* x, f4* y, bool vol = true) {
  bf4 xb[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) xb[i] = to_bf4(x[i]);
  matvec_b<OT, IT, HOIST, ACC>(W, ldw, xb, y, vol);
}
// the same product from operands already in bf16 (xb: T-layout tiles)
template <int OT, int IT, bool HOIST, bool ACC>
T2O_DEV void matvec_b(const __bf16* __restrict__ W, int ldw, const bf4* xb, f4* y, bool vol) {
  // HOIST false (T2O_SWZ_HOIST 0: the mixer BPTT kernels, register-bound at two
  // waves per SIMD): the lane's row swizzle is derived per product from an opaque
  // lane id, since hoisted out of the step loop one register per distinct row
  // length stays live (mixer BPTT spills 26 -> 4 VGPRs).  true (the agent
  // kernels and the mixer forward, which have registers to spare): computed
  // once, hoisted — per product it costs the agent ~7 % (interleaved A/B,
  // profiles/r3_ab_swz/).
  int l = threadIdx.x;
  if (!HOIST) asm volatile("" : "+v"(l));
  const int c = l & 15, g = (l >> 4) & 3;
  const int xs = bf_swz(c, ldw);
#pragma unroll
  for (int o = 0; o < OT; ++o) {
    const __bf16* row = W + (size_t)(16 * o + c) * ldw;
    f4 acc = ACC ? y[o] : zero4();
#pragma unroll
    for (int i = 0; i + 1 < IT; i += 2) {
      const __bf16* p0 = row + ((16 * i + 4 * g) ^ xs);
      const __bf16* p1 = row + ((16 * i + 16 + 4 * g) ^ xs);
      acc = mfma_b32(vol ? ldw4(p0) : ldb4(p0), vol ? ldw4(p1) : ldb4(p1), xb[i], xb[i + 1], acc);
    }
    if constexpr (IT & 1) {
      const __bf16* p = row + ((16 * (IT - 1) + 4 * g) ^ xs);
      acc = chain_tail_b16<(IT > 1)>(vol ? ldw4(p) : ldb4(p), xb[IT - 1], acc);
    }
    y[o] = acc;
  }
}

// The kernels' weight view: matrices (fp32 or bf16) and vectors (always fp32).
template <typename WT>
struct Wts {
  const WT* w;
  const float* v;
  // bf16: transposed products read the forward image transposed from LDS
  // (ds_read_b64_tr_b16) — else the pack's transposed copies (global memory, or
  // an LDS copy that includes them)
  bool tr;
  // bf16 weight fragments from LDS as volatile reads (ldw4) or plain ones the
  // compiler may fuse (ldb4); a compile-time constant of the kernel (it folds):
  // volatile pays in the two-wave-per-SIMD kernels, which are issue-bound;
  // the one-wave-per-SIMD kernels of 16+ entities and the one-wave multi-tile
  // mixer BPTT, latency-bound, measured slower with it (configs[0]-shape A/B,
  // profiles/r4_h16/: agent_bwd 1.67 -> 1.84 ms, mixer_bwd 3.62 -> 3.84 ms)
  bool vol = true;
  T2O_DEV float s(int64_t off) const { return (float)w[off]; }  // row 0 of a matrix (unswizzled row)
};

// y = Wᵀ x.  fp32 reads W transposed in place (matvec_t).  bf16 from LDS reads
// the forward image transposed with ds_read_b64_tr_b16: the A fragment of
// output tile o, K tile i is Wᵀ[16o + c][16i + 4g .. +3] = W[16i + 4g .. +3][16o + c],
// i.e. column 16o + c of the 4 rows 16i + 4g + q — exactly what the transposed
// read delivers to lane c of group g when lane 4q + p addresses row 16i + 4g + q,
// columns 16o + 4p .. +3.  The same bf16 values as the pack's transposed copy
// and the same K pairing, so the product is bit-identical to reading WT
// (which bf16 weights read through L2 still do).
template <int OT, int IT>
T2O_DEV void matvec_tr(const Wts<float>& P, int64_t off, int ld, int64_t offT, int ldT, const f4* x, f4* y);
T2O_DEV bf4 ld_tr_b16(const __bf16* p) {
  typedef __attribute__((address_space(3))) s4v lds_s4v;
  return __builtin_bit_cast(bf4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(p)));
}
template <int OT, int IT>
T2O_DEV void matvec_tr(const Wts<__bf16>& P, int64_t off, int ld, int64_t offT, int ldT, const f4* x, f4* y) {
  if (!P.tr) {
    matvec<OT, IT>(P.w + offT, ldT, x, y, P.vol);
    return;
  }
  // the lane's row q = 4g + (c >> 2) within a 16-row K tile and its column
  // offset, derived per product from an opaque lane id: hoisted out of the step
  // loop they would keep one register per matrix live
  int l = threadIdx.x;
  asm volatile("" : "+v"(l));
  const int c = l & 15, q = ((l >> 2) & 12) | (c >> 2);
  const int sw = bf_swz(q, ld);
  // (16o + 4p) ^ sw = (4p ^ (sw & 15)) + 16·(o ^ (sw >> 4)): the swizzle's low
  // bit permutes 4-element halves inside the lane's 8-element group, its high
  // bits permute whole 16-column output tiles
  const __bf16* W = P.w + off + q * ld + ((4 * (c & 3)) ^ (sw & 15));
  const int hi = sw >> 4;
  bf4 xb[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) xb[i] = to_bf4(x[i]);
#pragma unroll
  for (int o = 0; o < OT; ++o) {
    const int col = 16 * (o ^ hi);
    f4 acc = zero4();
#pragma unroll
    for (int i = 0; i + 1 < IT; i += 2)
      acc = mfma_b32(ld_tr_b16(W + (size_t)16 * i * ld + col), ld_tr_b16(W + (size_t)16 * (i + 1) * ld + col), xb[i],
                     xb[i + 1], acc);
    if constexpr (IT & 1) acc = chain_tail_b16<(IT > 1)>(ld_tr_b16(W + (size_t)16 * (IT - 1) * ld + col), xb[IT - 1], acc);
    y[o] = acc;
  }
}

// Weights staged in LDS are invariant across a kernel's step loop, so LICM
// would hoist every weight read out of the loop into registers (hundreds per
// lane, then spills).  Re-deriving the base pointer through an opaque zero
// offset at the top of each iteration keeps the reads as ds_reads at their use.
T2O_DEV const float* step_view(const float* base) {
  int off = 0;
  asm volatile("" : "+s"(off));
  return base + off;
}
template <typename WT>
T2O_DEV Wts<WT> step_view(const Wts<WT>& p) {
  int off = 0;
  asm volatile("" : "+s"(off));
  return Wts<WT>{p.w + off, p.v + off, p.tr, p.vol};
}

template <int OT, int IT>
T2O_DEV void matvec_tr(const Wts<float>& P, int64_t off, int ld, int64_t offT, int ldT, const f4* x, f4* y) {
  (void)offT;
  (void)ldT;
  matvec_t<OT, IT>(P.w + off, ld, x, y);
}

// T-layout slice of a bias / gamma vector: elements 16t+4g .. 16t+4g+3
T2O_DEV f4 vec_t(const float* __restrict__ v, int t) { return ld4(v + 16 * t + 4 * lane_g()); }

// ---- cross-lane reductions -------------------------------------------------
// Sum over the 4 lanes holding one row (c, c+16, c+32, c+48).  Additions are
// commutative pairings, so all four lanes get bit-identical results.
T2O_DEV float allsum4_shfl(float v) {
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}
T2O_DEV float allmax4_shfl(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  v = fmaxf(v, __shfl_xor(v, 32));
  return v;
}
// Sum over the 16 rows of a lane group (lanes 16g .. 16g+15).
T2O_DEV float rowsum16(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

// gfx950 VALU cross-lane forms (no LDS crossbar round trip).
// v_permlane16_swap: swaps rows 1,3 of the first operand with rows 0,2 of the
// second; with both operands = v the two results hold (v[l], v[l^16]) in some
// order, so their sum is the xor-16 pair sum.  permlane32_swap likewise for
// the two 32-lane halves.
T2O_DEV float xor16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
T2O_DEV float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
T2O_DEV float xor16_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
T2O_DEV float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
T2O_DEV float allsum4_fast(float v) { return xor32_sum(xor16_sum(v)); }
T2O_DEV float allmax4_fast(float v) { return xor32_max(xor16_max(v)); }
// the kernels' 4-lane all-reduces (bit-identical in the 4 lanes of a row)
T2O_DEV float allsum4(float v) { return allsum4_fast(v); }
T2O_DEV float allmax4(float v) { return allmax4_fast(v); }

// allsum4 of N independent values at once, in place, bit-identical to N
// allsum4 calls ((v_g0 + v_g1) + (v_g2 + v_g3) in every lane of the row).
// Values are reduced in fours: permlane16_swap(a, b) leaves (a, b) pair sums in
// alternating rows, permlane32_swap of two such registers leaves the four row
// totals one per row group ([A, B, C, D]), and three swaps broadcast them back
// — 12 VALU per 4 values instead of 24 (no copies needed in the reduction half
// since the operands are distinct).
T2O_DEV uint32_t f2u(float v) { return __float_as_uint(v); }
T2O_DEV float u2f(uint32_t v) { return __uint_as_float(v); }
T2O_DEV float pair_sum16(float a, float b) {  // [a01, b01, a23, b23]
  const auto r = __builtin_amdgcn_permlane16_swap(f2u(a), f2u(b), false, false);
  return u2f(r[0]) + u2f(r[1]);
}
template <int N>
T2O_DEV void allsum4_n(float (&v)[N]) {
  int i = 0;
#pragma unroll
  for (; i + 4 <= N; i += 4) {
    const float ab = pair_sum16(v[i], v[i + 1]), cd = pair_sum16(v[i + 2], v[i + 3]);
    const auto q = __builtin_amdgcn_permlane32_swap(f2u(ab), f2u(cd), false, false);
    const float w = u2f(q[0]) + u2f(q[1]);  // [A, B, C, D]
    const auto x = __builtin_amdgcn_permlane16_swap(f2u(w), f2u(w), false, false);  // [A,A,C,C], [B,B,D,D]
    const auto y = __builtin_amdgcn_permlane32_swap(x[0], x[0], false, false);      // [A..], [C..]
    const auto z = __builtin_amdgcn_permlane32_swap(x[1], x[1], false, false);      // [B..], [D..]
    v[i] = u2f(y[0]);
    v[i + 1] = u2f(z[0]);
    v[i + 2] = u2f(y[1]);
    v[i + 3] = u2f(z[1]);
  }
  if constexpr (N % 4 >= 2) {
    const float ab = pair_sum16(v[i], v[i + 1]);
    const auto q = __builtin_amdgcn_permlane32_swap(f2u(ab), f2u(ab), false, false);
    const float u = u2f(q[0]) + u2f(q[1]);  // [A, B, A, B]
    const auto x = __builtin_amdgcn_permlane16_swap(f2u(u), f2u(u), false, false);
    v[i] = u2f(x[0]);
    v[i + 1] = u2f(x[1]);
    i += 2;
  }
  if constexpr (N % 2) v[i] = allsum4(v[i]);
}

// The two halves of allsum4_n on their own.  rsum4_n: reduce-scatter, out[i] in
// lane group g = the row total of v[4i + g] (same pairing, so the same bits as
// allsum4 of that value) — a row's 4N values become N per lane, and elementwise
// work on them (a softmax over entities) runs once instead of in all 4 lanes.
// bcast4_n: the inverse, v[4i + k] = lane group k's in[i] in every lane.
template <int N>
T2O_DEV void rsum4_n(const float (&v)[4 * N], float (&out)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float ab = pair_sum16(v[4 * i], v[4 * i + 1]), cd = pair_sum16(v[4 * i + 2], v[4 * i + 3]);
    const auto q = __builtin_amdgcn_permlane32_swap(f2u(ab), f2u(cd), false, false);
    out[i] = u2f(q[0]) + u2f(q[1]);
  }
}
template <int N>
T2O_DEV void bcast4_n(const float (&in)[N], float (&v)[4 * N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const auto x = __builtin_amdgcn_permlane16_swap(f2u(in[i]), f2u(in[i]), false, false);
    const auto y = __builtin_amdgcn_permlane32_swap(x[0], x[0], false, false);
    const auto z = __builtin_amdgcn_permlane32_swap(x[1], x[1], false, false);
    v[4 * i] = u2f(y[0]);
    v[4 * i + 1] = u2f(z[0]);
    v[4 * i + 2] = u2f(y[1]);
    v[4 * i + 3] = u2f(z[1]);
  }
}

// Sum over the 16 lanes of a row with DPP (VALU only); the total lands in the
// row's last lane (c == 15) — other lanes hold partial sums.
template <int CTRL, int BANK>
T2O_DEV float dpp_shr(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, BANK, true));
}
T2O_DEV float rowsum16_fast(float v) {
  v += dpp_shr<0x111, 0xF>(v);   // row_shr:1
  v += dpp_shr<0x112, 0xF>(v);   // row_shr:2
  v += dpp_shr<0x114, 0xE>(v);   // row_shr:4, banks 1..3
  v += dpp_shr<0x118, 0xC>(v);   // row_shr:8, banks 2..3
  return v;
}

// log(1 + e) for e >= 0 (softplus), Goldberg's form: u = RN(1 + e) is exact
// as 1 + (u - 1), so log(u) · e / (u - 1) carries only the ~1 ulp relative errors
// of v_log_f32 (log2), the ln 2 product and v_rcp_f32; e itself where u rounds
// to 1.  (log(1 + e) alone lost up to 2^-24 / e relative to the rounding of 1 + e:
// 6e-5 at e = 2^-10, x·β near -7 — ADVICE r4.)  libm's log1pf / expf made a
// non-abs mixer head cost its kernels as much as the rest of the step (mixer
// BPTT 0.95 vs 0.54 ms).
T2O_DEV float log1p_fast(float e) {
  const float u = 1.f + e;
  const float um1 = u - 1.f;
  const float r = __builtin_amdgcn_logf(u) * 0.6931471805599453f * (e * rcp_fast(um1));
  return um1 == 0.f ? e : r;
}

// ---- mixing-head positivity (n_transf_mixer.py:95-103; the generic kernels) --
// pf = t2o_layout.pos_func (wave-uniform): abs, softplus(beta, torch's threshold
// 20), quadratic 0.5x², identity; dposf is the derivative torch's backward uses
// (abs: sign(x), 0 at 0).
T2O_DEV float posf(float x, int pf, float beta) {
  if (pf == T2O_POS_ABS) return fabsf(x);
  // (1/beta as v_rcp_f32: an IEEE division per call was a third of the head's work)
  if (pf == T2O_POS_SOFTPLUS) return x * beta > 20.f ? x : log1p_fast(exp_fast(x * beta)) * rcp_fast(beta);
  if (pf == T2O_POS_QUADRATIC) return 0.5f * x * x;
  return x;
}
T2O_DEV float dposf(float x, int pf, float beta) {
  if (pf == T2O_POS_ABS) return (float)((x > 0.f) - (x < 0.f));
  if (pf == T2O_POS_SOFTPLUS) {
    if (x * beta > 20.f) return 1.f;
    const float z = exp_fast(x * beta);
    return z * rcp_fast(z + 1.f);
  }
  if (pf == T2O_POS_QUADRATIC) return x;
  return 1.f;
}
// posf and dposf together (softplus: one exponential for both)
T2O_DEV void posd(float x, int pf, float beta, float& p, float& d) {
  if (pf == T2O_POS_SOFTPLUS) {
    if (x * beta > 20.f) {
      p = x;
      d = 1.f;
    } else {
      const float z = exp_fast(x * beta);
      p = log1p_fast(z) * rcp_fast(beta);
      d = z * rcp_fast(z + 1.f);
    }
    return;
  }
  p = posf(x, pf, beta);
  d = dposf(x, pf, beta);
}

// ---- LayerNorm over E = 16*ET features of each row (eps 1e-5, biased var) --
template <int ET>
T2O_DEV void layernorm_fwd(const f4* r, const float* __restrict__ gamma,
                           const float* __restrict__ beta, f4* out, f4* xhat, float& rstd) {
  constexpr float inv_e = 1.0f / (16 * ET);
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < ET; ++t) s += (r[t][0] + r[t][1]) + (r[t][2] + r[t][3]);
  const float mean = allsum4(s) * inv_e;
  float v = 0.f;
#pragma unroll
  for (int t = 0; t < ET; ++t) {
    const f4 d = r[t] - mean;
    v += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
  }
  const float var = allsum4(v) * inv_e;
  rstd = rsqrt_fast(var + 1e-5f);
#pragma unroll
  for (int t = 0; t < ET; ++t) {
    xhat[t] = (r[t] - mean) * rstd;
    out[t] = xhat[t] * vec_t(gamma, t) + vec_t(beta, t);
  }
}

// grad wrt LN input given grad wrt LN output (gamma applied inside)
template <int ET>
T2O_DEV void layernorm_bwd(const f4* gout, const f4* xhat, float rstd,
                           const float* __restrict__ gamma, f4* gin) {
  constexpr float inv_e = 1.0f / (16 * ET);
  f4 gx[ET];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int t = 0; t < ET; ++t) {
    gx[t] = gout[t] * vec_t(gamma, t);
    s1 += (gx[t][0] + gx[t][1]) + (gx[t][2] + gx[t][3]);
    const f4 p = gx[t] * xhat[t];
    s2 += (p[0] + p[1]) + (p[2] + p[3]);
  }
  float s[2] = {s1, s2};
  allsum4_n(s);
  const float m1 = s[0] * inv_e;
  const float m2 = s[1] * inv_e;
#pragma unroll
  for (int t = 0; t < ET; ++t) gin[t] = (gx[t] - m1 - xhat[t] * m2) * rstd;
}

}  // namespace t2o

namespace t2o {

// Cooperative copy of n floats (n % 4 == 0, 16-B aligned) global -> LDS by the whole block.
T2O_DEV void copy_to_lds(float* __restrict__ dst, const float* __restrict__ src, int64_t n) {
  for (int64_t i = 4 * (int64_t)threadIdx.x; i < n; i += 4 * (int64_t)blockDim.x) st4(dst + i, ld4(src + i));
}

// ---- a kernel's weight view ---------------------------------------------------
// fp32: the first n elements of the pack, copied as is.  bf16: the bf16 image of
// the first n elements (matrices; vector slots ride along unused) followed by
// the fp32 vector range [vec_lo, fwd_total).  Vectors are addressed with the
// pack's own offsets through a shifted base.  bf16: tr_reads (a compile-time
// constant at every call) — transposed products read the forward section
// transposed (matvec_tr), so n = fwd_total suffices; false: n = total also
// stages the pack's transposed copies, which they read instead.
T2O_DEV Wts<float> stage_weights(float* smem, const float* pack, const t2o_layout& L, int64_t n, float,
                                 bool = true) {
  copy_to_lds(smem, pack, n);
  return Wts<float>{smem, smem, false};
}
T2O_DEV Wts<__bf16> stage_weights(float* smem, const float* pack, const t2o_layout& L, int64_t n, __bf16,
                                  bool tr_reads = true) {
  copy_to_lds(smem, pack + L.total, n / 2);
  float* v = smem + n / 2;
  copy_to_lds(v, pack + L.vec_lo, L.fwd_total - L.vec_lo);
  return Wts<__bf16>{reinterpret_cast<const __bf16*>(smem), v - L.vec_lo, tr_reads};
}
T2O_DEV Wts<float> global_weights(const float* pack, const t2o_layout&, float) { return Wts<float>{pack, pack, false}; }
T2O_DEV Wts<__bf16> global_weights(const float* pack, const t2o_layout& L, __bf16) {
  return Wts<__bf16>{reinterpret_cast<const __bf16*>(pack + L.total), pack, false};
}
// LDS floats taken by stage_weights
template <typename WT>
__host__ __device__ inline int64_t lds_weight_floats(const t2o_layout& L, int64_t n) {
  return sizeof(WT) == 4 ? n : n / 2 + (L.fwd_total - L.vec_lo);
}

// Phase barrier of the two waves of one pipelined recurrence (the BPTT
// kernels' block-1 / block-0 wave pairs: an episode of the mixer, a 16-row tile
// of the agent).  Their only cross-wave dependencies run through the pair's
// own LDS region, so each wave writes a phase counter in LDS and polls its
// partner's instead of waiting for the whole workgroup: the other pairs' waves
// keep issuing while this pair waits (mixer BPTT 0.666 -> 0.652 ms).  Both waves
// of a pair must pass the same number of phases.  The wait is one inline-asm
// block (this wave's LDS ops drained, its counter written, the partner's polled
// with s_sleep between reads): a C++ spin loop kept values live across it and
// doubled the mixer kernel's register spills.  -DT2O_PIPE_WG_BARRIER:
// workgroup barriers instead (A/B).
constexpr int PAIR_FLAG_FLOATS = 16;  // LDS counters, one per wave (<= 16 waves)
#ifndef T2O_PAIR_SLEEP  // s_sleep argument between polls (64 cycles per unit)
#define T2O_PAIR_SLEEP 1
#endif
#define T2O_STR2(x) #x
#define T2O_STR(x) T2O_STR2(x)
struct PairBarrier {
  uint32_t mine, other;  // LDS byte addresses of the two counters (wave-uniform)
  int k;
  // counters at `flags` (zeroed before a workgroup barrier); partner = wave w ^ 1
  T2O_DEV static PairBarrier make(int* flags, int w) {
    typedef __attribute__((address_space(3))) int lds_int;
    const uint32_t fl = (uint32_t)(uintptr_t)(lds_int*)(flags);  // LDS byte address
    return PairBarrier{fl + 4u * w, fl + 4u * (w ^ 1), 0};
  }
  T2O_DEV void sync() {
#ifdef T2O_PIPE_WG_BARRIER
    __syncthreads();
#else
    ++k;
    int t;
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n\t"
        "ds_write_b32 %[a], %[kv]\n\t"
        "1:\n\t"
        "ds_read_b32 %[t], %[b]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_gt_i32 vcc, %[k], %[t]\n\t"
        "s_cbranch_vccz 2f\n\t"
        "s_sleep " T2O_STR(T2O_PAIR_SLEEP) "\n\t"
        "s_branch 1b\n"
        "2:"
        : [t] "=&v"(t)
        : [a] "v"(mine), [b] "v"(other), [kv] "v"(k), [k] "s"(k)
        : "vcc", "memory");
#endif
  }
};

// ---- weight-gradient accumulation -------------------------------------------
// dW[16*OT x 16*IT] += Σ_rows dY[row]ᵀ ⊗ X[row] over the wave's 16 rows, added
// into an LDS accumulator (row-major, leading dim ldw) with ds_add_f32.
// The contraction runs over ROWS, which the T-layout keeps on the lane axis,
// so both operands are transposed through a per-wave LDS staging area: the
// operand with fewer tiles is staged whole (row stride ≡ 16 mod 32 floats so
// the two 32-lane halves hit disjoint banks), the other is streamed one 16x16
// tile at a time.  MFMA step s consumes rows 4s..4s+3 (k = lane group g).
template <int NT>
struct StageDims {
  static constexpr int LD = 16 * NT + ((16 * NT) % 32 == 16 ? 0 : 16);  // ≡ 16 (mod 32)
  static constexpr int FLOATS = 16 * LD + 16 * 16;
};

T2O_DEV void stage_tile(float* st, int ld, int col0, f4 v) {
  *reinterpret_cast<f4*>(st + lane_c() * ld + col0 + 4 * lane_g()) = v;
}

template <int OT, int IT>
T2O_DEV void dw_accumulate(float* __restrict__ ldsW, int ldw, const f4* dY, const f4* X, float* stage) {
  constexpr int NS = OT < IT ? OT : IT;  // tiles staged whole
  constexpr int LD = StageDims<NS>::LD;
  float* st_full = stage;
  float* st_tile = stage + 16 * LD;
  const int c = lane_c(), g = lane_g();
  if constexpr (IT <= OT) {
#pragma unroll
    for (int i = 0; i < IT; ++i) stage_tile(st_full, LD, 16 * i, X[i]);
#pragma unroll
    for (int o = 0; o < OT; ++o) {
      stage_tile(st_tile, 16, 0, dY[o]);
      float a[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) a[s] = st_tile[(4 * s + g) * 16 + c];
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        f4 acc = zero4();
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(a[s], st_full[(4 * s + g) * LD + 16 * i + c], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(ldsW + (16 * o + 4 * g + r) * ldw + 16 * i + c, acc[r]);
      }
    }
  } else {
#pragma unroll
    for (int o = 0; o < OT; ++o) stage_tile(st_full, LD, 16 * o, dY[o]);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      stage_tile(st_tile, 16, 0, X[i]);
      float bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) bv[s] = st_tile[(4 * s + g) * 16 + c];
#pragma unroll
      for (int o = 0; o < OT; ++o) {
        f4 acc = zero4();
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(st_full[(4 * s + g) * LD + 16 * o + c], bv[s], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(ldsW + (16 * o + 4 * g + r) * ldw + 16 * i + c, acc[r]);
      }
    }
  }
}

// bf16 staging tiles of the register-block contractions: tile j of a wave's
// stage is [16 rows][16 features] bf16; a lane writes its T-layout f4 (row c,
// features 4g..4g+3: one 8-byte store) and reads back the K-slice over rows
// (feature c of rows 4g..4g+3) with one ds_read_b64_tr_b16.  Row r keeps its
// four 8-byte chunks in the order chunk ^ ((r >> 2) & 3): the 16 writes of a
// lane group (rows 0..15, one chunk) then cover 32 distinct store banks
// (unswizzled: 4-way), and every transposed read still takes whole 32-B rows.
T2O_DEV void stage_tile_bf(__bf16* sb, int j, f4 v) {
  const int c = lane_c(), g = lane_g();
  *reinterpret_cast<bf4*>(sb + j * 256 + c * 16 + 4 * (g ^ ((c >> 2) & 3))) = to_bf4(v);
}
T2O_DEV bf4 kslice_tile_bf(const __bf16* sb, int j) {
  typedef __attribute__((address_space(3))) s4v lds_s4v;
  const int c = lane_c(), g = lane_g();
  const __bf16* p = sb + j * 256 + (4 * g + (c >> 2)) * 16 + 4 * ((c & 3) ^ g);
  return __builtin_bit_cast(bf4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(p)));
}

// acc[o][i] += Σ_rows dY[o] ⊗ X[i] with X already staged (stage_tile_bf) in
// tiles xt .. xt+IT-1 of the wave's stage — e.g. by an earlier phase of the
// same wave — and dY streamed through tile yt.
template <int OT, int IT>
T2O_DEV void dw_accumulate_prestaged(f4 (&acc)[OT][IT], const f4* dY, float* stage, int xt, int yt) {
  __bf16* sb = reinterpret_cast<__bf16*>(stage);
  bf4 xb[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) xb[i] = kslice_tile_bf(sb, xt + i);
#pragma unroll
  for (int o = 0; o < OT; ++o) {
    stage_tile_bf(sb, yt, dY[o]);
    asm volatile("" ::: "memory");
    const bf4 ab = kslice_tile_bf(sb, yt);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < IT; ++i) acc[o][i] = mfma_b16(ab, xb[i], acc[o][i]);
  }
}

// Same contraction, accumulated into MFMA accumulator registers acc[o][i]
// (a wave-private gradient block that stays in registers across calls).
// BF: bf16 operands, one 16x16x16 MFMA over the 16 rows per tile pair.
template <int OT, int IT, bool BF = false>
T2O_DEV void dw_accumulate_regs(f4 (&acc)[OT][IT], const f4* dY, const f4* X, float* stage) {
  constexpr int NS = OT < IT ? OT : IT;
  const int c = lane_c(), g = lane_g();
  if constexpr (BF) {
    // bf16: operand tiles are staged as [16 rows][16 features] bf16 (one
    // 8-byte write per lane) and read back transposed with one
    // ds_read_b64_tr_b16 — lane (g, c) gets feature c of rows 4g..4g+3, the
    // 16x16x16 K-slice over rows.  The X side is staged whole, dY one tile at
    // a time (so the stage holds IT + 1 tiles).  Row r keeps its four 8-byte
    // chunks in the order chunk ^ ((r >> 2) & 3): the 16 writes of a lane group
    // (rows 0..15, one chunk) then cover 32 distinct store banks (unswizzled:
    // 4-way), and every transposed read still takes whole 32-B rows.
    static_assert((IT + 1) * 128 <= StageDims<NS>::FLOATS, "stage too small");
    __bf16* sb = reinterpret_cast<__bf16*>(stage);
#pragma unroll
    for (int i = 0; i < IT; ++i) stage_tile_bf(sb, 1 + i, X[i]);
    bf4 xb[IT];
#pragma unroll
    for (int o = 0; o < OT; ++o) {
      stage_tile_bf(sb, 0, dY[o]);
      asm volatile("" ::: "memory");  // a wave's LDS accesses complete in order; keep the compiler's order too
      if (o == 0) {
#pragma unroll
        for (int i = 0; i < IT; ++i) xb[i] = kslice_tile_bf(sb, 1 + i);
      }
      const bf4 ab = kslice_tile_bf(sb, 0);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < IT; ++i) acc[o][i] = mfma_b16(ab, xb[i], acc[o][i]);
    }
    return;
  }
  // fp32: the side with fewer tiles is staged whole (row stride ≡ 16 mod 32
  // floats), the other streamed one 16x16 tile at a time; MFMA step s consumes
  // rows 4s..4s+3 (k = lane group g)
  constexpr int LD = StageDims<NS>::LD;
  float* st_full = stage;
  float* st_tile = stage + 16 * LD;
  if constexpr (IT <= OT) {
#pragma unroll
    for (int i = 0; i < IT; ++i) stage_tile(st_full, LD, 16 * i, X[i]);
#pragma unroll
    for (int o = 0; o < OT; ++o) {
      stage_tile(st_tile, 16, 0, dY[o]);
      float a[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) a[s] = st_tile[(4 * s + g) * 16 + c];
#pragma unroll
      for (int i = 0; i < IT; ++i)
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[o][i] = mfma4(a[s], st_full[(4 * s + g) * LD + 16 * i + c], acc[o][i]);
    }
  } else {
#pragma unroll
    for (int o = 0; o < OT; ++o) stage_tile(st_full, LD, 16 * o, dY[o]);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      stage_tile(st_tile, 16, 0, X[i]);
      float bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) bv[s] = st_tile[(4 * s + g) * 16 + c];
#pragma unroll
      for (int o = 0; o < OT; ++o)
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[o][i] = mfma4(st_full[(4 * s + g) * LD + 16 * o + c], bv[s], acc[o][i]);
    }
  }
}

// vec[16*NT] += Σ_rows v[row]  (T-layout input; one lane per group adds)
template <int NT>
T2O_DEV void vec_accumulate(float* __restrict__ ldsv, const f4* v) {
  const int c = lane_c(), g = lane_g();
  float s[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) s[t][r] = rowsum16_fast(v[t][r]);  // total in lane c == 15
  if (c == 15) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(ldsv + 16 * t + 4 * g + r, s[t][r]);
  }
}


// Same sum into a global (per-workgroup slab) vector with hardware float
// atomics (no return value, fire-and-forget at L2).
template <int NT>
T2O_DEV void vec_accumulate_g(float* __restrict__ gv, const f4* v) {
  const int c = lane_c(), g = lane_g();
  float s[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) s[t][r] = rowsum16_fast(v[t][r]);
  if (c == 15) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) unsafeAtomicAdd(gv + 16 * t + 4 * g + r, s[t][r]);
  }
}

// Zero the parts of a workgroup's gradient slab (compact layout, grad_layout)
// that its BPTT kernel flushes into: the head region (We, be, Wo, bo), every
// block's LN2 vectors and, when the tape does not carry their operands (lean
// agent record), every block's M and N.  The tape contraction (t2o_dwgemm.hip)
// overwrites every other region of every slab it owns with plain stores, so
// zeroing the whole slab (grad_total floats per workgroup: 86 MB per agent BPTT
// at configs[2]) only added HBM writes.  All threads of the workgroup take part;
// the caller's barrier follows.
T2O_DEV void zero_flushed_regions(float* __restrict__ gs, const t2o_layout& G, bool mn) {
  const int nt = (int)blockDim.x;
  for (int i = threadIdx.x; i < (int)G.M[0]; i += nt) gs[i] = 0.f;  // We, be, Wo, bo
  for (int d = 0; d < G.D; ++d) {
    for (int i = threadIdx.x; i < 2 * G.E; i += nt) gs[G.g2[d] + i] = 0.f;  // g2, n2 (adjacent)
    if (mn)
      for (int i = threadIdx.x; i < 2 * G.H * G.E * G.E; i += nt) gs[G.M[d] + i] = 0.f;  // M, N (adjacent)
  }
}

// Deterministic end-of-kernel slab flush: the workgroup's waves add their
// partial sums into the workgroup's slab one wave at a time, in wave order —
// wave w's float atomics are performed at L2 (s_waitcnt) before the barrier that
// lets wave w + 1 issue — so every slab element receives its addends in the same
// order on every run (concurrent waves' atomics would not, and the update would
// not be bit-reproducible).  Within a wave each flush touches an element at most
// once.  Every wave of the workgroup must call this exactly once.
template <typename F>
T2O_DEV void flush_in_wave_order(F&& flush) {
#ifdef T2O_NONDET_FLUSH  // A/B builds only: concurrent flushes (not bit-reproducible)
  flush();
  return;
#endif
  const int nw = (int)(blockDim.x >> 6);
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  for (int turn = 0; turn < nw; ++turn) {
    if (turn == w) {
      flush();
      __builtin_amdgcn_s_waitcnt(0);
    }
    __syncthreads();
  }
}

// Flush an MFMA-layout register block acc[o][i] (lane (g,c), reg r holds
// dW[16o+4g+r][16i+c]) into a global row-major matrix with float atomics.
template <int OT, int IT>
T2O_DEV void flush_tiles_g(float* __restrict__ W, int ldw, const f4 (&acc)[OT][IT]) {
  const int c = lane_c(), g = lane_g();
#pragma unroll
  for (int o = 0; o < OT; ++o)
#pragma unroll
    for (int i = 0; i < IT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) unsafeAtomicAdd(W + (16 * o + 4 * g + r) * ldw + 16 * i + c, acc[o][i][r]);
}

// ---- weight-gradient tape ---------------------------------------------------
// The backward kernels do not accumulate the four big per-block matrices
// (M, N, W1, W2), nor the FFN / LN1 / unify vectors, themselves: per (row,
// step, block) they stream a record to an HBM tape, and t2o_dwgemm.hip
// contracts the tape over all records with MFMA:
//   dM = Σ gu ⊗ x,  dN = Σ gres ⊗ z,  dW2 = Σ gr2 ⊗ relu(f1),  P = Σ gf1 ⊗ x̂1,
//   d bu = Σ gres,  d c2 = Σ gr2,  d c1 = Σ gf1,  Q = Σ gr2 ⊙ x̂1
// with y = x̂1 ⊙ g1 + n1, f1 = W1 y + c1 and gf1 = [f1 > 0] ⊙ W2ᵀ gr2
// RECOMPUTED by the contraction from (x̂1, gr2).  The LN1 output y and its grad
// gy = gr2 + W1ᵀ gf1 are not stored: every quantity they fed is linear in them,
// so t2o_unpack_grads completes the three affected grads from the summed slab
// (T_UNFOLD_LN1, t2o_pack.hip):
//   dW1 = Σ gf1 ⊗ y = P ⊙ g1 + d c1 ⊗ n1
//   d g1 = Σ gy ⊙ x̂1 = Q + Σ_J W1[J] ⊙ P[J]
//   d n1 = Σ gy = d c2 + W1ᵀ d c1
// Only the LN2 vectors (g2, n2) and the small embedding / head grads are still
// summed inside the backward kernels.  Feature offsets of one record:
template <int E, int H, int FF>
struct TapeRec {
  static constexpr int X = 0;                 // block input x      (E)   M:  X
  static constexpr int GU = X + E;            // dL/du              (HE)  M:  dY
  static constexpr int Z = GU + H * E;        // head outputs z     (HE)  N:  X
  static constexpr int GRES = Z + H * E;      // dL/d(N z + bu)     (E)   N:  dY, bu
  static constexpr int GR2 = GRES + E;        // dL/d(W2 f + c2 + y)(E)   W2: dY, gf1, c2, Q
  static constexpr int XH1 = GR2 + E;         // LN1 x̂             (E)   y, P, Q
  static constexpr int SIZE = XH1 + E;
};

// The agent's pipelined bf16 BPTT accumulates dM and dN in registers
// (dw_accumulate_prestaged) and tapes only the rest: the lean agent record.
// X, GU, Z are absent (negative offsets).
template <int E, int H, int FF>
struct TapeRecA {
  static constexpr int X = -1, GU = -1, Z = -1;
  static constexpr int GRES = 0;
  static constexpr int GR2 = GRES + E;
  static constexpr int XH1 = GR2 + E;
  static constexpr int SIZE = XH1 + E;
};

// Layout: tiles of 16 records (one wave's rows at one step), RECORD-major
// inside a tile: element (record 16·tile + c, feature f) of block d sits at
// ((d·ntiles + tile)·16 + c)·SIZE + f, in the MFMA operand type (fp32, or
// bf16 in bf16 mode).  A writer lane (g, c) holds features 16t + 4g .. +3 of
// record c, i.e. 8 (bf16) / 16 (fp32) contiguous bytes: one store per 16
// features.  The contraction stages whole tiles in LDS and reads the
// feature-major K-slices of its MFMAs with the gfx950 transposed LDS read.

// store a T-layout vector (NT tiles, features off + 16t + 4g + r of record c)
template <int SIZE, int NT, typename TT>
T2O_DEV void rec_store(TT* __restrict__ tile, int off, const f4* v) {
  TT* p = tile + lane_c() * SIZE + off + 4 * lane_g();
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if constexpr (sizeof(TT) == 2) {
      *reinterpret_cast<bf4*>(p + 16 * t) = to_bf4(v[t]);
    } else {
      st4(reinterpret_cast<float*>(p + 16 * t), v[t]);
    }
  }
}

// A tape tile written through a buffer resource: lanes whose record lies at or
// past `rows` get an out-of-range offset and the buffer unit drops their
// stores, so a tile of fewer than 16 records needs no per-lane branch (exec-mask
// control flow around every store costs registers in the two-wave kernels).
// The tile base must be wave-uniform.
// CPOL: cache policy of the tape stores (the buffer instructions' aux bits; 2 =
// non-temporal).  Interleaved A/B (profiles/r3_cpol/, r3_shp/): nt cut the
// multi-tile mixer BPTT at 32 AGVs 8.16 -> 7.32 ms and left the one-tile
// pipelined mixer and the agent kernels unchanged in time while their PMC write
// bytes rose 18-39 % (partial-line nt writes), so only the multi-tile mixer uses
// it; write-through (sc1) was slower everywhere (update 2.506 -> 2.598 ms).
template <typename TT, int CPOL = 0>
struct MaskedRec {
  __amdgpu_buffer_rsrc_t rsrc;
  int voff;  // bytes: this lane's record, features 4g.. ; or out of range
  T2O_DEV MaskedRec(TT* tile, int rows, int size) {
    const uint64_t a = reinterpret_cast<uint64_t>(tile);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    TT* base = reinterpret_cast<TT*>(((uint64_t)hi << 32) | lo);
    rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, rows * size * (int)sizeof(TT), 0x00020000);
    voff = lane_c() < rows ? (lane_c() * size + 4 * lane_g()) * (int)sizeof(TT) : 0x40000000;
  }
  // a T-layout vector (NT tiles): features off + 16t + 4g + r of this lane's record
  template <int NT>
  T2O_DEV void store(int off, const f4* v) const {
    typedef int v2i __attribute__((ext_vector_type(2)));
    typedef int v4i __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int o = voff + (off + 16 * t) * (int)sizeof(TT);
      if constexpr (sizeof(TT) == 2) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, to_bf4(v[t])), rsrc, o, 0, CPOL);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v[t]), rsrc, o, 0, CPOL);
      }
    }
  }
};

}  // namespace t2o
