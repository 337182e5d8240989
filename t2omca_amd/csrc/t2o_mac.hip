// t2o_mac.hip — ε-greedy action selection of the multi-agent controller on
// the device, closing the rollout loop env -> agent -> env
// without the per-step host round trip of parallel_runner.py:121-122.
//
// The reference's controller / action selector modules are absent;
// the contract is mac.select_actions(batch, t_ep, t_env, bs, test_mode)
// (parallel_runner.py:121) with PyMARL's EpsilonGreedyActionSelector:
//   masked_q = q with unavailable actions at -inf; pick_random = u1 < ε;
//   random action ~ Categorical(avail) (uniform over the available actions);
//   action = pick_random ? random : argmax(masked_q)   (first maximum wins).
// The two uniforms of (row, step) are the counter-based stream of
// env_spec.uniforms (t2o_env.hip): u1 = U(seed, row, 2·counter),
// u2 = U(seed, row, 2·counter + 1), and the random action is the
// floor(u2 · n_avail)-th available one — so oracle/ref_mac.py reproduces every
// draw exactly.
#include "t2o_common.hpp"

namespace {

// the selector's own stream: seed keyed with T2O_STREAM_MAC (t2o_common.hpp), so
// exploration draws never repeat the env's dynamics draws of the same row
__device__ double mac_uniform(uint64_t seed, int64_t row, int64_t idx) {
  uint64_t x = ((uint64_t)row << 40) | (uint64_t)idx;
  x ^= (seed ^ T2O_STREAM_MAC) * 0xD1B54A32D192ED03ull;
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (double)(z >> 11) * 0x1.0p-53;
}

constexpr int MAC_MAXNA = 32;

__global__ void select_actions_kernel(const float* __restrict__ q, const int32_t* __restrict__ avail,
                                      int64_t* __restrict__ actions, int64_t rows, int NA, double eps,
                                      uint64_t seed, int64_t counter) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float* qr = q + r * NA;
  const int32_t* ar = avail + r * NA;
  int best = 0, navail = 0;
  float bq = -INFINITY;
  bool any = false;
  for (int k = 0; k < NA; ++k) {
    const bool ok = ar[k] != 0;
    navail += ok;
    const float v = ok ? qr[k] : -INFINITY;
    if (!any || v > bq) {
      bq = v;
      best = k;
      any = true;
    }
  }
  int act = best;
  if (eps > 0.0) {
    const double u1 = mac_uniform(seed, r, 2 * counter);
    if (u1 < eps && navail > 0) {
      const double u2 = mac_uniform(seed, r, 2 * counter + 1);
      int kth = (int)(u2 * (double)navail);
      if (kth >= navail) kth = navail - 1;
      for (int k = 0; k < NA; ++k) {
        if (ar[k] != 0) {
          if (kth == 0) {
            act = k;
            break;
          }
          --kth;
        }
      }
    }
  }
  actions[r] = act;
}

}  // namespace

extern "C" int t2o_select_actions(const float* q, const int32_t* avail, int64_t* actions, int64_t rows, int NA,
                                  double epsilon, uint64_t seed, int64_t counter, void* stream) {
  if (!q || !avail || !actions || rows < 0 || NA < 1 || NA > MAC_MAXNA || counter < 0) return T2O_EINVAL;
  if (rows == 0) return 0;
  const int64_t blocks = (rows + 255) / 256;
  hipLaunchKernelGGL(select_actions_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, q, avail,
                     actions, rows, NA, epsilon, seed, counter);
  return (int)hipGetLastError();
}
