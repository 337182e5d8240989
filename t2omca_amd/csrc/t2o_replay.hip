// t2o_replay.hip — device-resident prioritized episode replay.
//
// The reference's buffer module is absent (components.episode_buffer,
// SURVEY §0); its contract is per_run.py:143-146 (PrioritizedReplayBuffer(
// scheme, groups, buffer_size, episode_limit + 1, per_alpha, per_beta, t_max))
// and :216-238 (insert_episode_batch, can_sample, sample(batch, t_env) ->
// (batch, idx, weights), update_priorities(idx, td_errors_abs + 1e-6)) with
// PyMARL2's proportional PER semantics:
//   stored priority      p_i = priority_i ^ alpha   (new episodes: max_priority ^ alpha)
//   stratified sampling  mass_k = (u_k + k) · Σp / batch,  idx_k = min{i : Σ_{j<=i} p_j > mass_k}
//   IS weights           w_k = (p_idx / Σp · N) ^ -beta / (p_min / Σp · N) ^ -beta
// Here the sum / min segment trees become one prefix scan per sample (one
// workgroup; a replay of a few thousand episodes is a few µs), the uniforms are
// the counter-based stream of env_spec.uniforms (u_k = U(seed, k, counter)),
// and the sampled episodes are gathered into a dense batch by a byte-granular
// gather kernel (one launch per stored tensor).
#include "t2o_common.hpp"

namespace {

// PER's draws are their own stream: the seed is keyed with a per-stream constant
// (env: none, MAC: T2O_STREAM_MAC, PER: T2O_STREAM_PER), so replay sampling never
// repeats the env's or the action selector's draws for the same seed.
__device__ double per_uniform(uint64_t seed, int64_t row, int64_t idx) {
  uint64_t x = ((uint64_t)row << 40) | (uint64_t)idx;
  x ^= (seed ^ T2O_STREAM_PER) * 0xD1B54A32D192ED03ull;
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (double)(z >> 11) * 0x1.0p-53;
}

constexpr int PER_THREADS = 1024;

// One workgroup: inclusive prefix sum of p[0..n) (fp64) into cum, the minimum,
// then batch threads binary-search their stratified mass.
__global__ __launch_bounds__(PER_THREADS) void per_sample_kernel(const float* __restrict__ p, int64_t n,
                                                                 int64_t batch, double beta, uint64_t seed,
                                                                 int64_t counter, double* __restrict__ cum,
                                                                 int64_t* __restrict__ idx_out,
                                                                 float* __restrict__ w_out) {
  __shared__ double part[PER_THREADS];
  __shared__ float pmin_s[PER_THREADS];
  const int tid = threadIdx.x;
  const int64_t chunk = (n + PER_THREADS - 1) / PER_THREADS;
  const int64_t lo = tid * chunk, hi = lo + chunk < n ? lo + chunk : n;
  double s = 0.0;
  float mn = INFINITY;
  for (int64_t i = lo; i < hi; ++i) {
    s += (double)p[i];
    mn = fminf(mn, p[i]);
  }
  part[tid] = s;
  pmin_s[tid] = mn;
  __syncthreads();
  // Hillis-Steele inclusive scan of the per-thread sums (fixed order: deterministic)
  for (int off = 1; off < PER_THREADS; off <<= 1) {
    const double v = tid >= off ? part[tid - off] : 0.0;
    const float m = tid >= off ? pmin_s[tid - off] : INFINITY;
    __syncthreads();
    part[tid] += v;
    pmin_s[tid] = fminf(pmin_s[tid], m);
    __syncthreads();
  }
  double run = tid > 0 ? part[tid - 1] : 0.0;
  for (int64_t i = lo; i < hi; ++i) {
    run += (double)p[i];
    cum[i] = run;
  }
  __syncthreads();
  const double total = part[PER_THREADS - 1];
  const double pmin = (double)pmin_s[PER_THREADS - 1];
  const double max_w = pow(pmin / total * (double)n, -beta);
  for (int64_t k = tid; k < batch; k += PER_THREADS) {
    const double mass = (per_uniform(seed, k, counter) + (double)k) * (total / (double)batch);
    int64_t a = 0, b = n - 1;  // smallest i with cum[i] > mass
    while (a < b) {
      const int64_t mid = (a + b) / 2;
      if (cum[mid] > mass) b = mid;
      else a = mid + 1;
    }
    idx_out[k] = a;
    w_out[k] = (float)(pow((double)p[a] / total * (double)n, -beta) / max_w);
  }
}

__global__ void per_update_kernel(float* __restrict__ p, const int64_t* __restrict__ idx,
                                  const float* __restrict__ prio, int64_t n, float alpha, float eps,
                                  float* __restrict__ max_prio) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const float v = prio[k] + eps;
  // PyMARL2 asserts priority > 0; a non-positive or non-finite value (a NaN's bit
  // pattern would win the unsigned max below for good) leaves the episode as it was
  if (!(v > 0.f) || !isfinite(v)) return;
  p[idx[k]] = powf(v, alpha);
  atomicMax(reinterpret_cast<unsigned int*>(max_prio), __float_as_uint(v));  // v > 0: bit order = value order
}

// dst[k] = src[idx[k]] for rows of row_units units of U bytes
template <typename U>
__global__ void gather_rows_kernel(const char* __restrict__ src, int64_t src_stride, const int64_t* __restrict__ idx,
                                   int64_t rows, char* __restrict__ dst, int64_t dst_stride, int64_t row_units) {
  const int64_t k = blockIdx.y;
  if (k >= rows) return;
  const U* s = reinterpret_cast<const U*>(src + idx[k] * src_stride);
  U* d = reinterpret_cast<U*>(dst + k * dst_stride);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < row_units; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

}  // namespace

extern "C" int64_t t2o_per_workspace_doubles(int64_t capacity) { return capacity < 1 ? 1 : capacity; }

extern "C" int t2o_per_sample(const float* p, int64_t n, int64_t batch, double beta, uint64_t seed, int64_t counter,
                              double* workspace, int64_t* idx_out, float* w_out, void* stream) {
  if (!p || !workspace || !idx_out || !w_out || n < 1 || batch < 1 || counter < 0 || counter >= (1ll << 40) ||
      batch >= (1ll << 24))
    return T2O_EINVAL;
  hipLaunchKernelGGL(per_sample_kernel, dim3(1), dim3(PER_THREADS), 0, (hipStream_t)stream, p, n, batch, beta, seed,
                     counter, workspace, idx_out, w_out);
  return (int)hipGetLastError();
}

extern "C" int t2o_per_update(float* p, const int64_t* idx, const float* prio, int64_t n, float alpha, float eps,
                              float* max_prio, void* stream) {
  if (!p || !idx || !prio || !max_prio || n < 0) return T2O_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(per_update_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, p, idx,
                     prio, n, alpha, eps, max_prio);
  return (int)hipGetLastError();
}

extern "C" int t2o_gather_rows(const void* src, int64_t src_stride, const int64_t* idx, int64_t rows, void* dst,
                               int64_t dst_stride, int64_t row_bytes, void* stream) {
  if (!src || !idx || !dst || rows < 0 || row_bytes < 0 || rows > 65535) return T2O_EINVAL;
  if (rows == 0 || row_bytes == 0) return 0;
  // widest unit every address and size is a multiple of
  const uint64_t al = (uint64_t)reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) |
                      (uint64_t)src_stride | (uint64_t)dst_stride | (uint64_t)row_bytes;
  const int unit = (al % 16 == 0) ? 16 : (al % 8 == 0) ? 8 : (al % 4 == 0) ? 4 : 1;
  const int64_t units = row_bytes / unit;
  int64_t bx = (units + 255) / 256;
  if (bx > 64) bx = 64;
  const dim3 grid((unsigned)bx, (unsigned)rows);
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  switch (unit) {
    case 16: hipLaunchKernelGGL(gather_rows_kernel<uint4>, grid, dim3(256), 0, (hipStream_t)stream, s, src_stride, idx,
                                rows, d, dst_stride, units); break;
    case 8: hipLaunchKernelGGL(gather_rows_kernel<uint2>, grid, dim3(256), 0, (hipStream_t)stream, s, src_stride, idx,
                               rows, d, dst_stride, units); break;
    case 4: hipLaunchKernelGGL(gather_rows_kernel<uint32_t>, grid, dim3(256), 0, (hipStream_t)stream, s, src_stride,
                               idx, rows, d, dst_stride, units); break;
    default: hipLaunchKernelGGL(gather_rows_kernel<uint8_t>, grid, dim3(256), 0, (hipStream_t)stream, s, src_stride,
                                idx, rows, d, dst_stride, units); break;
  }
  return (int)hipGetLastError();
}
