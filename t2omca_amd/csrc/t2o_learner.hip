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
  const void* term;       // [B][T] strides tm_sb, tm_st (0/1, element type tm_dt)
  const void* filled;     // [B][T] strides fl_sb, fl_st (0/1, element type fl_dt)
  const float* weight;    // [B] or null
  int64_t rw_sb, rw_st, tm_sb, tm_st, fl_sb, fl_st;
  float gamma, lambda_;
  float mask_sum;         // > 0: use this global Σ mask (data parallel); else local
  float* gq;              // [B][T]  dL/dQtot
  float* targets;         // [B][T]  (may be null)
  float* prio;            // [B]
  float* loss;            // [2]: loss, Σ mask
  float* mask_acc;        // optional: += Σ mask (the learner's grad[-1] slot)
  int B, T;
  int tm_dt, fl_dt;       // T2O_DT_* (t2omca.h): the EpisodeBatch's own dtypes, read in place
};

// one 0/1 mask element of the given storage type as float
__device__ float mask_at(const void* p, int64_t i, int dt) {
  switch (dt) {
    case T2O_DT_U8: return (float)static_cast<const uint8_t*>(p)[i];
    case T2O_DT_I32: return (float)static_cast<const int32_t*>(p)[i];
    case T2O_DT_I64: return (float)static_cast<const int64_t*>(p)[i];
    default: return static_cast<const float*>(p)[i];
  }
}

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

// Episodes are independent: a workgroup stages EP episodes' rows in LDS with
// coalesced loads, one thread per episode runs the (sequential, as in the
// reference) backward TD(λ) recursion out of LDS, and the block writes gq /
// targets back coalesced.  Loss and Σ mask are accumulated with float atomics
// into loss[] (zeroed by the host entry); with mask_sum <= 0 a second pass
// divides gq and the loss by the local Σ mask.
//   mask[b][t] = filled[t] * (t == 0 ? 1 : 1 - term[t-1])   (PyMARL2 nq_learner)
__global__ __launch_bounds__(256) void td_loss_kernel(TDArgs a, int EP) {
  extern __shared__ float sm[];
  T2O_LDS_POISON(sm);
  __shared__ float red[8];
  const int T = a.T;
  const int b0 = blockIdx.x * EP;
  const int nb = min(EP, a.B - b0);
  float* R = sm;                 // reward, then dL/dQtot
  float* TM = R + EP * T;        // terminated
  float* FL = TM + EP * T;       // filled, then targets
  float* Q = FL + EP * T;        // qtot
  float* QT = Q + EP * T;        // qtot_tgt [EP][T+1]
  for (int i = threadIdx.x; i < nb * T; i += blockDim.x) {
    const int b = b0 + i / T, t = i % T;
    R[i] = a.reward[b * a.rw_sb + t * a.rw_st];
    TM[i] = a.term ? mask_at(a.term, b * a.tm_sb + t * a.tm_st, a.tm_dt) : 0.f;
    FL[i] = a.filled ? mask_at(a.filled, b * a.fl_sb + t * a.fl_st, a.fl_dt) : 1.f;
    Q[i] = a.qtot[(size_t)b0 * T + i];
  }
  for (int i = threadIdx.x; i < nb * (T + 1); i += blockDim.x) QT[i] = a.qtot_tgt[(size_t)b0 * (T + 1) + i];
  __syncthreads();
  const float denom = a.mask_sum > 0.f ? a.mask_sum : 1.f;
  float lsum = 0.f, msum = 0.f;
  if ((int)threadIdx.x < nb) {
    const int e = threadIdx.x, b = b0 + e;
    const float* r = R + e * T;
    const float* tm = TM + e * T;
    const float* fl = FL + e * T;
    const float* q = Q + e * T;
    const float* qt = QT + e * (T + 1);
    // build_td_lambda_targets: ret[T] = Q[T] * (1 - Σ term); backwards recursion
    float tsum = 0.f;
    for (int t = 0; t < T; ++t) tsum += tm[t];
    float ret = qt[T] * (1.f - tsum);
    const float w = a.weight ? a.weight[b] : 1.f;
    float absum = 0.f, mb = 0.f, lb = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      const float m = fl[t] * (t > 0 ? 1.f - tm[t - 1] : 1.f);
      ret = a.lambda_ * a.gamma * ret + m * (r[t] + (1.f - a.lambda_) * a.gamma * qt[t + 1] * (1.f - tm[t]));
      const float td = q[t] - ret;
      // in-place: row t of R / FL is not read again
      R[e * T + t] = w * m * td / denom;
      FL[e * T + t] = ret;
      absum += fabsf(td) * m;
      mb += m;
      lb += 0.5f * td * td * m;
    }
    a.prio[b] = mb > 0.f ? absum / sqrtf(mb) : 0.f;  // an all-masked episode: 0, not 0/0
    lsum = lb * w;
    msum = mb;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb * T; i += blockDim.x) {
    a.gq[(size_t)b0 * T + i] = R[i];
    if (a.targets) a.targets[(size_t)b0 * T + i] = FL[i];
  }
  lsum = block_sum(lsum, red);
  msum = block_sum(msum, red);
  if (threadIdx.x == 0) {
    unsafeAtomicAdd(a.loss, lsum / denom);
    unsafeAtomicAdd(a.loss + 1, msum);
    if (a.mask_acc) unsafeAtomicAdd(a.mask_acc, msum);
  }
}

// The same targets / loss / priorities with one WAVE per episode: the TD(λ)
// recursion ret_t = λγ·ret_{t+1} + B_t (B_t = m_t (r_t + (1-λ)γ Q'_{t+1}(1-term_t)),
// B_T = Q'_T (1 - Σ term)) is linear with a constant multiplier, so lane l takes
// the chunk [lC, lC + C) of t = 0..T (C = ⌈(T+1)/64⌉), folds it from its end
// (G_l, P_l = λγ^len), a Hillis–Steele suffix scan of (G, P) pairs across the
// wave gives each chunk its incoming ret, and a second pass over the chunk
// re-runs the recursion from it.  Reassociated (fp32 rounding differs from the
// sequential order by ~1e-7 relative), deterministic, and the T-step serial
// chain becomes C + 6 steps.
constexpr int TDW_WAVES = 4;

__global__ __launch_bounds__(64 * TDW_WAVES) void td_loss_wave_kernel(TDArgs a) {
  __shared__ float red[2][TDW_WAVES];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x * TDW_WAVES + w;
  const int T = a.T;
  const float A = a.lambda_ * a.gamma, G1 = (1.f - a.lambda_) * a.gamma;
  const float denom = a.mask_sum > 0.f ? a.mask_sum : 1.f;
  float lsum = 0.f, msum = 0.f;
  if (b < a.B) {
    const int C = (T + 1 + 63) / 64;
    const int t0 = min(lane * C, T + 1), t1 = min(t0 + C, T + 1);
    auto tm = [&](int t) { return a.term ? mask_at(a.term, (int64_t)b * a.tm_sb + (int64_t)t * a.tm_st, a.tm_dt) : 0.f; };
    auto fl = [&](int t) { return a.filled ? mask_at(a.filled, (int64_t)b * a.fl_sb + (int64_t)t * a.fl_st, a.fl_dt) : 1.f; };
    const float* qt = a.qtot_tgt + (size_t)b * (T + 1);
    float ts = 0.f;
    for (int t = t0; t < t1 && t < T; ++t) ts += tm(t);
    for (int o = 32; o > 0; o >>= 1) ts += __shfl_xor(ts, o);
    auto mask = [&](int t) { return fl(t) * (t > 0 ? 1.f - tm(t - 1) : 1.f); };
    auto Bt = [&](int t) {
      if (t == T) return qt[T] * (1.f - ts);
      return mask(t) * (a.reward[(int64_t)b * a.rw_sb + (int64_t)t * a.rw_st] + G1 * qt[t + 1] * (1.f - tm(t)));
    };
    float g = 0.f, p = 1.f;
    for (int t = t1 - 1; t >= t0; --t) {
      g = Bt(t) + A * g;
      p *= A;
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const float gd = __shfl_down(g, d), pd = __shfl_down(p, d);
      if (lane + d < 64) {
        g = g + p * gd;
        p = p * pd;
      }
    }
    float ret = __shfl_down(g, 1);
    if (lane == 63) ret = 0.f;
    const float wb = a.weight ? a.weight[b] : 1.f;
    float absum = 0.f, mb = 0.f, lb = 0.f;
    for (int t = t1 - 1; t >= t0; --t) {
      ret = Bt(t) + A * ret;
      if (t == T) continue;
      const float m = mask(t);
      const float td = a.qtot[(size_t)b * T + t] - ret;
      a.gq[(size_t)b * T + t] = wb * m * td / denom;
      if (a.targets) a.targets[(size_t)b * T + t] = ret;
      absum += fabsf(td) * m;
      mb += m;
      lb += 0.5f * td * td * m;
    }
    for (int o = 32; o > 0; o >>= 1) {
      absum += __shfl_xor(absum, o);
      mb += __shfl_xor(mb, o);
      lb += __shfl_xor(lb, o);
    }
    if (lane == 0) a.prio[b] = mb > 0.f ? absum / sqrtf(mb) : 0.f;  // an all-masked episode: 0, not 0/0
    lsum = lb * wb;
    msum = mb;
  }
  if (lane == 0) {
    red[0][w] = lsum;
    red[1][w] = msum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float l = 0.f, m = 0.f;
    for (int i = 0; i < TDW_WAVES; ++i) {
      l += red[0][i];
      m += red[1][i];
    }
    unsafeAtomicAdd(a.loss, l / denom);
    unsafeAtomicAdd(a.loss + 1, m);
    if (a.mask_acc) unsafeAtomicAdd(a.mask_acc, m);
  }
}

// mask_sum <= 0: normalise by the local Σ mask once it is complete.
__global__ __launch_bounds__(256) void td_normalise_kernel(float* __restrict__ gq, int64_t n, float* loss) {
  const float inv = 1.0f / loss[1];  // (PyMARL2: / mask.sum())
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    gq[i] *= inv;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) loss[0] *= inv;  // the grid has one block
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

static int td_impl(const float* qtot, const float* qtot_tgt, const float* reward, int64_t rw_sb,
                               int64_t rw_st, const void* term, int term_dtype, int64_t tm_sb, int64_t tm_st,
                               const void* filled, int filled_dtype, int64_t fl_sb, int64_t fl_st,
                               const float* per_weight, float gamma, float td_lambda, float mask_sum, float* gq,
                               float* targets, float* prio, float* loss, float* mask_sum_acc, int algo, int B,
                               int T, void* stream) {
  if (!qtot || !qtot_tgt || !reward || !gq || !prio || !loss || B < 1 || T < 1) return T2O_EINVAL;
  auto dt_ok = [](int dt) { return dt == T2O_DT_F32 || dt == T2O_DT_U8 || dt == T2O_DT_I32 || dt == T2O_DT_I64; };
  if (!dt_ok(term_dtype) || !dt_ok(filled_dtype)) return T2O_EINVAL;
  if (algo < T2O_TD_AUTO || algo > T2O_TD_WAVE_SCAN) return T2O_EINVAL;
  TDArgs a{qtot, qtot_tgt, reward, term, filled, per_weight, rw_sb, rw_st, tm_sb, tm_st, fl_sb, fl_st,
           gamma, td_lambda, mask_sum, gq, targets, prio, loss, mask_sum_acc, B, T, term_dtype, filled_dtype};
  hipStream_t s = (hipStream_t)stream;
  // AUTO = the wave scan: 8-10 us faster per configs[2] update than the sequential
  // kernel (interleaved, profiles/r4_a/), parity equal (tests/test_gpu_td_loss.py)
  const bool wave = algo != T2O_TD_SEQUENTIAL;
  if (hipMemsetAsync(loss, 0, 2 * sizeof(float), s) != hipSuccess) return (int)hipGetLastError();
  if (wave) {
    hipLaunchKernelGGL(td_loss_wave_kernel, dim3((B + TDW_WAVES - 1) / TDW_WAVES), dim3(64 * TDW_WAVES), 0, s, a);
  } else {
    const size_t per_ep = sizeof(float) * (5 * (size_t)T + 1);
    // episodes per workgroup: few enough that the grid covers the CUs (the
    // staging loads, not the per-episode scan, dominate a fat workgroup)
    int ep = (int)((96 * 1024) / per_ep);
    if (ep > 64) ep = 64;
    const int ep_fill = (B + 255) / 256;
    if (ep > ep_fill) ep = ep_fill;
    if (ep < 1) return T2O_EUNSUPPORTED;  // T beyond the LDS staging (> ~4900 steps): use the wave scan
    (void)hipFuncSetAttribute((const void*)td_loss_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(ep * per_ep));
    hipLaunchKernelGGL(td_loss_kernel, dim3((B + ep - 1) / ep), dim3(256), ep * per_ep, s, a, ep);
  }
  if (mask_sum <= 0.f)
    hipLaunchKernelGGL(td_normalise_kernel, dim3(1), dim3(256), 0, s, gq, (int64_t)B * T, loss);
  return (int)hipGetLastError();
}

extern "C" int t2o_td_loss(const t2o_td_args* a, void* stream) {
  if (!a) return T2O_EINVAL;
  return td_impl(a->qtot, a->qtot_tgt, a->reward, a->rw_sb, a->rw_st, a->term, a->term_dtype, a->tm_sb, a->tm_st,
                 a->filled, a->filled_dtype, a->fl_sb, a->fl_st, a->per_weight, a->gamma, a->td_lambda, a->mask_sum,
                 a->gq, a->targets, a->prio, a->loss, a->mask_sum_acc, a->algo, a->B, a->T, stream);
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
