// t2o_probe.hip — on-device checks of the cross-lane primitives the kernels use
// (semantics of DPP row reductions, gfx950 permlane swaps and the batched
// all-reduce are verified by
// tests/test_gpu_primitives.py against host-computed expectations).
#include "t2o_common.hpp"

using namespace t2o;

namespace {
__global__ void probe_kernel(const float* __restrict__ in, float* __restrict__ out) {
  const int l = threadIdx.x;
  const float v = in[l];
  out[0 * 64 + l] = allsum4_shfl(v);
  out[1 * 64 + l] = allsum4_fast(v);
  out[2 * 64 + l] = rowsum16(v);
  out[3 * 64 + l] = rowsum16_fast(v);
  out[4 * 64 + l] = allmax4_shfl(v);
  out[5 * 64 + l] = allmax4_fast(v);
  // batched all-reduce (7 = one group of four, a pair, a single) vs one at a time
  float b[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) b[k] = in[(l + 9 * k) % 64] * (float)(k + 1);
#pragma unroll
  for (int k = 0; k < 7; ++k) out[(13 + k) * 64 + l] = allsum4(b[k]);
  allsum4_n(b);
#pragma unroll
  for (int k = 0; k < 7; ++k) out[(6 + k) * 64 + l] = b[k];
}
}  // namespace

extern "C" int t2o_probe_lane_ops(const float* in, float* out, void* stream) {
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, in, out);
  return (int)hipGetLastError();
}

// The mixing head's positivity functions (posf / dposf / the fused posd the
// BPTT kernels call) element by element, for a per-element check against torch
// (tests/test_gpu_primitives.py; n_transf_mixer.py:95-103).
namespace {
__global__ void probe_posf_kernel(const float* __restrict__ x, int n, int pf, float beta, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  float p, d;
  posd(v, pf, beta, p, d);
  out[i] = posf(v, pf, beta);
  out[n + i] = dposf(v, pf, beta);
  out[2 * n + i] = p;
  out[3 * n + i] = d;
}
}  // namespace

extern "C" int t2o_probe_posf(const float* x, int n, int pos_func, float beta, float* out, void* stream) {
  if (!x || !out || n < 0) return T2O_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(probe_posf_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, n, pos_func,
                     beta, out);
  return (int)hipGetLastError();
}

// The reduce-scatter / broadcast halves of the batched all-reduce (the agent's
// scattered softmax), the packed 4-feature dot product, and the 8-wide bf16
// conversion with the bit-pattern ReLU (tests/test_gpu_primitives.py).
// out rows: 0-1 rsum4_n of 8 values, 2-9 bcast4_n of them, 10-17 allsum4_n of the
// same 8 values, 18 dot4_pk, 19-22 relu_bf8(cvt8(a, b)) as packed bf16 words.
namespace {
__global__ void probe_scatter_kernel(const float* __restrict__ in, float* __restrict__ out) {
  const int l = threadIdx.x;
  float v[8], a8[8], r[2], bc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = a8[k] = in[(l + 5 * k) % 64] * (float)(k + 1);
  rsum4_n(v, r);
  bcast4_n(r, bc);
  allsum4_n(a8);
#pragma unroll
  for (int k = 0; k < 2; ++k) out[k * 64 + l] = r[k];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    out[(2 + k) * 64 + l] = bc[k];
    out[(10 + k) * 64 + l] = a8[k];
  }
  const f4 x{in[l], in[(l + 1) % 64], in[(l + 2) % 64], in[(l + 3) % 64]};
  const f4 y{in[(l + 17) % 64], in[(l + 29) % 64], in[(l + 41) % 64], in[(l + 53) % 64]};
  out[18 * 64 + l] = dot4_pk(x, y);
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const u4 w = __builtin_bit_cast(u4, relu_bf8(cvt8(x, y)));
#pragma unroll
  for (int k = 0; k < 4; ++k) out[(19 + k) * 64 + l] = __uint_as_float(w[k]);
}
}  // namespace

extern "C" int t2o_probe_scatter_ops(const float* in, float* out, void* stream) {
  if (!in || !out) return T2O_EINVAL;
  hipLaunchKernelGGL(probe_scatter_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, in, out);
  return (int)hipGetLastError();
}

// MFMA result hand-offs with a FIXED number of wait states, written in inline asm
// so the compiler's hazard recognizer neither pads nor reorders them
// (tests/test_gpu_primitives.py::test_xdl_hand_off_wait_states):
// each variant computes an MFMA into a[0:3] and hands the result on after the
// given number of wait states; the compiler-padded builtin computes the reference.
//   0 / 1  v_mfma_f32_16x16x4_f32 -> ds_write_b128 of its AGPRs after 10 / 32 states
//   2 / 3  v_mfma_f32_16x16x4_f32 -> global_store_dwordx4 of its AGPRs after 10 / 32
//   4 / 5 / 6  v_mfma_f32_16x16x32_bf16 -> v_mfma_f32_16x16x16_bf16 reading its result
//          as srcC after 0 / 4 / 32 states (the odd key-tile pairing's chain)
//   7 / 8  one opcode's chain, 16x16x32 -> 16x16x32, after 0 / 32 states
// then three compiler-built references (the same products through the builtins,
// hazards padded by hipcc): the f32 MFMA, the mixed chain, the one-opcode chain.
// 10 states is what hipcc (ROCm 7.2) leaves between such a 16x16x4 f32 result and
// an LDS or VMEM store of it; 0-4 what it leaves before a dependent srcC read of
// another opcode.  32 states is past any MFMA's latency: the ground truth.
namespace {
constexpr int XP_VARIANTS = 9;
#define XP_LOAD_C                          \
  "s_nop 4\n\t"                            \
  "v_accvgpr_write_b32 a0, %[c0]\n\t"      \
  "v_accvgpr_write_b32 a1, %[c1]\n\t"      \
  "v_accvgpr_write_b32 a2, %[c2]\n\t"      \
  "v_accvgpr_write_b32 a3, %[c3]\n\t"      \
  "s_nop 7\n\t"
#define XP_C_IN [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3])

__global__ __launch_bounds__(64) void probe_xdl_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                      int nwaves) {
  __shared__ f4 lds[2][64];
  const int l = threadIdx.x, w = blockIdx.x;
  const float* src = in + ((size_t)w * 64 + l) * 12;
  const float a = src[0], b = src[1];
  const f4 c{src[2], src[3], src[4], src[5]};
  const bf8 a8 = cvt8(f4{src[6], src[7], src[8], src[9]}, f4{src[10], src[11], src[0], src[1]});
  const bf8 b8 = cvt8(f4{src[11], src[10], src[9], src[8]}, f4{src[7], src[6], src[5], src[4]});
  const bf4 a4 = to_bf4(f4{src[3], src[2], src[1], src[0]}), b4 = to_bf4(f4{src[4], src[6], src[8], src[10]});
  float* o = out + ((size_t)w * 64 + l) * 4;
  const size_t vs = (size_t)nwaves * 64 * 4;  // one variant's block
  auto put = [&](int v, f4 r) { *reinterpret_cast<f4*>(o + v * vs) = r; };
  // references (hazards padded by the compiler)
  put(XP_VARIANTS, mfma4(a, b, c));
  put(XP_VARIANTS + 1, mfma_b16(a4, b4, __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c, 0, 0, 0)));
  put(XP_VARIANTS + 2, __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                           a8, b8, __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c, 0, 0, 0), 0, 0, 0));
  typedef __attribute__((address_space(3))) f4 lds_f4;
  const uint32_t la0 = (uint32_t)(uintptr_t)(lds_f4*)(&lds[0][l]), la1 = (uint32_t)(uintptr_t)(lds_f4*)(&lds[1][l]);
  asm volatile(XP_LOAD_C
               "v_mfma_f32_16x16x4_f32 a[0:3], %[a], %[b], a[0:3]\n\t"
               "s_nop 9\n\t"
               "ds_write_b128 %[addr], a[0:3]\n\t"
               "s_waitcnt lgkmcnt(0)"
               :: XP_C_IN, [a] "v"(a), [b] "v"(b), [addr] "v"(la0) : "a0", "a1", "a2", "a3", "memory");
  asm volatile(XP_LOAD_C
               "v_mfma_f32_16x16x4_f32 a[0:3], %[a], %[b], a[0:3]\n\t"
               "s_nop 15\n\ts_nop 15\n\t"
               "ds_write_b128 %[addr], a[0:3]\n\t"
               "s_waitcnt lgkmcnt(0)"
               :: XP_C_IN, [a] "v"(a), [b] "v"(b), [addr] "v"(la1) : "a0", "a1", "a2", "a3", "memory");
  __builtin_amdgcn_wave_barrier();
  put(0, lds[0][l]);
  put(1, lds[1][l]);
  float* g2 = o + 2 * vs;
  float* g3 = o + 3 * vs;
  asm volatile(XP_LOAD_C
               "v_mfma_f32_16x16x4_f32 a[0:3], %[a], %[b], a[0:3]\n\t"
               "s_nop 9\n\t"
               "global_store_dwordx4 %[p], a[0:3], off\n\t"
               "s_waitcnt vmcnt(0)"
               :: XP_C_IN, [a] "v"(a), [b] "v"(b), [p] "v"(g2) : "a0", "a1", "a2", "a3", "memory");
  asm volatile(XP_LOAD_C
               "v_mfma_f32_16x16x4_f32 a[0:3], %[a], %[b], a[0:3]\n\t"
               "s_nop 15\n\ts_nop 15\n\t"
               "global_store_dwordx4 %[p], a[0:3], off\n\t"
               "s_waitcnt vmcnt(0)"
               :: XP_C_IN, [a] "v"(a), [b] "v"(b), [p] "v"(g3) : "a0", "a1", "a2", "a3", "memory");
  f4 r;
#define XP_CHAIN(SECOND, PAD)                                                                             \
  asm volatile(XP_LOAD_C                                                                                  \
               "v_mfma_f32_16x16x32_bf16 a[0:3], %[a8], %[b8], a[0:3]\n\t" PAD SECOND                    \
               "s_nop 15\n\ts_nop 15\n\t"                                                                 \
               "v_accvgpr_read_b32 %[r0], a0\n\t"                                                         \
               "v_accvgpr_read_b32 %[r1], a1\n\t"                                                         \
               "v_accvgpr_read_b32 %[r2], a2\n\t"                                                         \
               "v_accvgpr_read_b32 %[r3], a3\n\t"                                                         \
               "s_nop 4"                                                                                  \
               : [r0] "=v"(r[0]), [r1] "=v"(r[1]), [r2] "=v"(r[2]), [r3] "=v"(r[3])                     \
               : XP_C_IN, [a8] "v"(a8), [b8] "v"(b8), [a4] "v"(a4), [b4] "v"(b4)                         \
               : "a0", "a1", "a2", "a3")
#define XP_16 "v_mfma_f32_16x16x16_bf16 a[0:3], %[a4], %[b4], a[0:3]\n\t"
#define XP_32 "v_mfma_f32_16x16x32_bf16 a[0:3], %[a8], %[b8], a[0:3]\n\t"
#define XP_PAD32 "s_nop 15\n\ts_nop 15\n\t"
  XP_CHAIN(XP_16, "");
  put(4, r);
  XP_CHAIN(XP_16, "s_nop 3\n\t");
  put(5, r);
  XP_CHAIN(XP_16, XP_PAD32);
  put(6, r);
  XP_CHAIN(XP_32, "");
  put(7, r);
  XP_CHAIN(XP_32, XP_PAD32);
  put(8, r);
#undef XP_CHAIN
#undef XP_16
#undef XP_32
#undef XP_PAD32
}
#undef XP_LOAD_C
#undef XP_C_IN
}  // namespace

// out: [XP_VARIANTS + 3][nwaves][64][4] floats (the variants, then the f32, the
// mixed-chain and the same-opcode-chain references); in: [nwaves][64][12] floats
extern "C" int t2o_probe_xdl_hazards(const float* in, float* out, int nwaves, void* stream) {
  if (!in || !out || nwaves < 1) return T2O_EINVAL;
  hipLaunchKernelGGL(probe_xdl_kernel, dim3(nwaves), dim3(64), 0, (hipStream_t)stream, in, out, nwaves);
  return (int)hipGetLastError();
}
