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
