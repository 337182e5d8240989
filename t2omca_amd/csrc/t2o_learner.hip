// t2o_learner.hip — TD targets / loss / priorities and the clipped Adam step.
//
// The reference ships no learner: per_run.py:224-238 only fixes the contract
//   info = learner.train(batch, t_env, episode, per_weights)
//   buffer.update_priorities(idx, info["td_errors_abs"].flatten() + 1e-6)
// These kernels implement the PyMARL2 NQLearner semantics that contract comes
// from (parity-unpinned beyond the agent/mixer arithmetic):
//   targets  = build_td_lambda_targets(r, term, mask, Qtot_tgt[0..T], γ, λ)
//   td       = Qtot[0..T-1] - targets
//   loss     = Σ_b w_b Σ_t ½ td² m / Σ m
//   prio_b   = Σ_t |td| m / √(Σ_t m)
// and torch.nn.utils.clip_grad_norm_ + torch.optim.Adam (non-amsgrad, L2
// weight decay) on the flat parameter buffer.
#include <math.h>

#include "t2o_common.hpp"

namespace {

struct TDArgs {
  const float* qtot;      // [B][T]
  const float* qtot_tgt;  // [B][T+1]
  const float* reward;    // [B][T] strides rw_sb, rw_st
  const float* term;      // [B][T] strides tm_sb, tm_st (float 0/1)
  const float* filled;    // [B][T] strides fl_sb, fl_st (float 0/1)
  const float* weight;    // [B] or null
  int64_t rw_sb, rw_st, tm_sb, tm_st, fl_sb, fl_st;
  float gamma, lambda_;
  float mask_sum;         // > 0: use this global Σ mask (data parallel); else local
  float* gq;              // [B][T]  dL/dQtot
  float* targets;         // [B][T]  (may be null)
  float* prio;            // [B]
  float* loss;            // [2]: loss, Σ mask
  int B, T;
};

__device__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

// mask[b][t] = filled[t] * (t == 0 ? 1 : 1 - term[t-1])   (PyMARL2 nq_learner)
__device__ float mask_at(const TDArgs& a, int b, int t) {
  float m = a.filled ? a.filled[b * a.fl_sb + t * a.fl_st] : 1.f;
  if (t > 0 && a.term) m *= 1.f - a.term[b * a.tm_sb + (t - 1) * a.tm_st];
  return m;
}

__global__ __launch_bounds__(1024) void td_loss_kernel(TDArgs a) {
  __shared__ float red[16];
  const int T = a.T;
  float msum = 0.f;
  for (int b = threadIdx.x; b < a.B; b += blockDim.x)
    for (int t = 0; t < T; ++t) msum += mask_at(a, b, t);
  const float local_msum = block_sum(msum, red);
  const float denom = a.mask_sum > 0.f ? a.mask_sum : local_msum;
  float lsum = 0.f;
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    // build_td_lambda_targets: ret[T] = Q[T] * (1 - Σ term); backwards recursion
    float tsum = 0.f;
    if (a.term)
      for (int t = 0; t < T; ++t) tsum += a.term[b * a.tm_sb + t * a.tm_st];
    float ret = a.qtot_tgt[(size_t)b * (T + 1) + T] * (1.f - tsum);
    const float w = a.weight ? a.weight[b] : 1.f;
    float absum = 0.f, mb = 0.f, lb = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      const float m = mask_at(a, b, t);
      const float r = a.reward[b * a.rw_sb + t * a.rw_st];
      const float tm = a.term ? a.term[b * a.tm_sb + t * a.tm_st] : 0.f;
      ret = a.lambda_ * a.gamma * ret +
            m * (r + (1.f - a.lambda_) * a.gamma * a.qtot_tgt[(size_t)b * (T + 1) + t + 1] * (1.f - tm));
      if (a.targets) a.targets[(size_t)b * T + t] = ret;
      const float td = a.qtot[(size_t)b * T + t] - ret;
      a.gq[(size_t)b * T + t] = w * m * td / denom;
      absum += fabsf(td) * m;
      mb += m;
      lb += 0.5f * td * td * m;
    }
    a.prio[b] = absum / sqrtf(mb);
    lsum += lb * w;
  }
  const float tot = block_sum(lsum, red);
  if (threadIdx.x == 0) {
    a.loss[0] = tot / denom;
    a.loss[1] = local_msum;
  }
}

// ---- Adam -------------------------------------------------------------------
constexpr int NORM_BLOCKS = 256;

__global__ __launch_bounds__(256) void sqnorm_partials(const float* __restrict__ g, int64_t n,
                                                       float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += g[i] * g[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

struct AdamArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  const float* part;  // NORM_BLOCKS partial Σ g² (null: no clipping)
  const float* gdiv;  // [1] optional device divisor applied to every grad (data-parallel Σ mask)
  float* norm_out;    // [1] grad norm before clipping (may be null)
  int64_t n;
  float omb1, beta2, omb2, eps, weight_decay, max_norm;  // 1-β1, β2, 1-β2 (rounded from double)
  float step_size;    // lr / (1 - β1^step)
  float bc2_sqrt;     // sqrt(1 - β2^step)
};

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  const float inv = a.gdiv ? 1.0f / a.gdiv[0] : 1.0f;
  float coef = inv;
  if (a.part) {
    float s = 0.f;
    for (int i = 0; i < NORM_BLOCKS; ++i) s += a.part[i];
    const float norm = sqrtf(s) * inv;
    coef = inv * fminf(a.max_norm / (norm + 1e-6f), 1.0f);
    if (a.norm_out && blockIdx.x == 0 && threadIdx.x == 0) a.norm_out[0] = norm;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    float g = a.g[i] * coef;
    float p = a.p[i];
    if (a.weight_decay != 0.f) g += a.weight_decay * p;
    float m = a.m[i];
    m = m + (g - m) * a.omb1;            // exp_avg.lerp_(grad, 1 - beta1)
    float v = a.v[i] * a.beta2 + g * g * a.omb2;
    a.m[i] = m;
    a.v[i] = v;
    const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
    a.p[i] = p - a.step_size * (m / denom);
  }
}

}  // namespace

extern "C" int t2o_td_loss(const float* qtot, const float* qtot_tgt, const float* reward, int64_t rw_sb,
                           int64_t rw_st, const float* term, int64_t tm_sb, int64_t tm_st, const float* filled,
                           int64_t fl_sb, int64_t fl_st, const float* per_weight, float gamma, float td_lambda,
                           float mask_sum, float* gq, float* targets, float* prio, float* loss, int B, int T,
                           void* stream) {
  if (!qtot || !qtot_tgt || !reward || !gq || !prio || !loss || B < 1 || T < 1) return T2O_EINVAL;
  TDArgs a{qtot, qtot_tgt, reward, term, filled, per_weight, rw_sb, rw_st, tm_sb, tm_st, fl_sb, fl_st,
           gamma, td_lambda, mask_sum, gq, targets, prio, loss, B, T};
  hipLaunchKernelGGL(td_loss_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

extern "C" int t2o_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                             float* workspace, int64_t n, double lr, double beta1, double beta2, float eps,
                             float weight_decay, float max_grad_norm, int64_t step, const float* grad_div,
                             float* grad_norm_out, void* stream) {
  if (!params || !grads || !exp_avg || !exp_avg_sq || n < 1 || step < 1) return T2O_EINVAL;
  if (max_grad_norm > 0.f && !workspace) return T2O_EINVAL;
  AdamArgs a{};
  a.p = params;
  a.g = grads;
  a.m = exp_avg;
  a.v = exp_avg_sq;
  a.n = n;
  a.omb1 = (float)(1.0 - beta1);
  a.beta2 = (float)beta2;
  a.omb2 = (float)(1.0 - beta2);
  a.eps = eps;
  a.weight_decay = weight_decay;
  a.max_norm = max_grad_norm;
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  a.step_size = (float)(lr / bc1);
  a.bc2_sqrt = (float)sqrt(bc2);
  a.norm_out = grad_norm_out;
  a.gdiv = grad_div;
  hipStream_t s = (hipStream_t)stream;
  if (max_grad_norm > 0.f) {
    hipLaunchKernelGGL(sqnorm_partials, dim3(NORM_BLOCKS), dim3(256), 0, s, grads, n, workspace);
    a.part = workspace;
  }
  int blocks = (int)((n + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

extern "C" int t2o_adam_workspace_floats(void) { return NORM_BLOCKS; }
