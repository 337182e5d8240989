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
