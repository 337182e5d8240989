// t2o_env.hip — vectorised MultiAgvOffloadingEnv on MI355X (one wave per env).
//
// Reference: environment_multi_mec.py (step :309-366, get_reward :229-293,
// calculate_offload_delay :106-121, get_agent_inf :123-146, get_obs_agent
// :148-182, get_obs :184-186, get_state :188-204, reset/reset_user
// :206-227, update_users :295-307, get_avail_agent_actions :61-74) and
// normalization.py:4-35, driven with parallel_runner.py's worker protocol
// (:239-263).  Stand-in constants and the counter-based draw stream:
// t2omca_amd/env_spec.py (mirrored in EnvSpec below).
//
// Exactness.  Decisions (bincount collisions, acks, avail masks, job queues,
// indices) are integer work and bit-exact.  The float path is IEEE fp64 with
// FMA contraction OFF so every +,-,*,/,sqrt rounds as numpy/CPython do; the
// reference's two rounding flavours are reproduced exactly:
//   numpy   round(np.float64, 2) = rint(x*100)/100
//   CPython round(float, 2)      = correctly rounded decimal (exact x*100 via fma)
// Only log10/log2/pow come from the device libm (ocml) instead of glibc; their
// results pass through a 2-decimal rounding before anything observable, and
// tests/test_gpu_env.py measures agreement with the numpy oracle.
#pragma clang fp contract(off)
#include <math.h>

#include "t2o_common.hpp"

namespace {

struct EnvSpec {
  double mec_radius, comp_cycles, bandwidth, noise, path_loss, cgl, mec_cap, tx_power, user_cap;
  int latency_max, t_length, size_min, size_max;
  double arrival_p;
  int edge_only;  // get_avail_agent_actions' edge_only variant (:63-68)
  int obs_entity;  // obs_entity_mode (:148-182): 1 entity obs [A][9A], 0 flat [A][6]
};

// get_obs_agent's length: entity mode 9 features per entity, else
// [last_ack, get_agent_inf(5)] (:172-182); the normaliser has the same length (:59)
__host__ __device__ inline int obs_len(int obs_entity, int A) { return obs_entity ? 9 * A : 6; }

struct EnvState {
  int32_t* mec_index;   // [NE][A]
  double* x;            // [NE][A]
  double* y;
  int32_t* q_size;      // [NE][A][QMAX]
  int32_t* q_thr;       // [NE][A][QMAX]
  int32_t* q_head;      // [NE][A]
  int32_t* q_len;       // [NE][A]
  int32_t* task_num;    // [NE][A]
  int32_t* task_success;
  double* remain_delay;
  int32_t* last_ack;    // [NE][A]
  int32_t* time_slot;   // [NE]
  int64_t* draw;        // [NE]
  int64_t* nrm_n;       // [NE]
  double* nrm_mean;     // [NE][9A]
  double* nrm_S;
  double* nrm_std;
};

struct EnvOut {
  float* obs;           // [NE][A][9A] (may be null)
  double* obs64;        // [NE][A][9A] (may be null)
  float* state;         // [NE][8A] (may be null)
  int32_t* avail;       // [NE][A][nA] (may be null)
  double* reward;       // [NE]
  uint8_t* terminated;  // [NE]
  double* info;         // [NE][6]: delay_reward, overtime, utilization, conflict_ratio,
                        //          task_completion_rate, task_completion_delay (NaN if not terminal)
  int32_t* ack;         // [NE][A]
  // compact observation wire format, written beside (or instead
  // of) the dense obs by every get_obs whose result the worker returns:
  int32_t* wire;        // [NE][A][4] (may be null), see WIRE_* below
  int64_t* snap_n;      // [NE]  normaliser count before the worker's get_obs in reset
  double* snap;         // [NE][2][9A] normaliser mean, S at the same point
};

struct EnvArgs {
  EnvSpec sp;
  EnvState s;
  EnvOut o;
  const int64_t* actions;  // [NE][A] (step)
  int64_t act_se;          // element stride between envs
  int NE, A, M, C, QMAX, T;
  uint64_t seed;
  int mode;                // 0 init, 1 reset, 2 step, 3 env_info
  int apad, G;             // lane map (lane_map): agent lanes per env, envs per wave
};

constexpr int MAXA = 64;

// ---- counter-based uniforms (env_spec.uniforms) -----------------------------
__device__ __forceinline__ double uniform(uint64_t seed, int env, int64_t idx) {
  uint64_t x = ((uint64_t)env << 40) | (uint64_t)idx;
  x ^= seed * 0xD1B54A32D192ED03ull;
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (double)(z >> 11) * 0x1.0p-53;
}

__device__ __forceinline__ double round2_numpy(double x) { return rint(x * 100.0) / 100.0; }

// CPython round(x, 2): round-half-even of the EXACT value x*100, then /100.
__device__ __forceinline__ double round2_python(double x) {
  const double p = x * 100.0;
  const double e = fma(x, 100.0, -p);  // exact: x*100 = p + e
  double r = rint(p);
  const double fl = floor(p);
  if (p - fl == 0.5) {  // p is a half-integer: the exact value decides
    if (e > 0.0) r = fl + 1.0;
    else if (e < 0.0) r = fl;
  }
  return r / 100.0;
}

__device__ __forceinline__ void mec_pos(const EnvArgs& a, int m, double& mx, double& my) {
  mx = (double)m * (a.sp.mec_radius * 2) + a.sp.mec_radius;
  my = a.sp.mec_radius;
}

__device__ __forceinline__ void position(const EnvArgs& a, int m, double u1, double u2, double& x, double& y) {
  double mx, my;
  mec_pos(a, m, mx, my);
  const double aa = 2.0 * u1 - 1.0;
  const double bb = 2.0 * u2 - 1.0;
  x = mx + a.sp.mec_radius * aa;
  y = my + (a.sp.mec_radius * bb) * sqrt(1.0 - aa * aa);
}

// calculate_offload_delay (:106-121)
__device__ __forceinline__ double offload_delay(const EnvArgs& a, int mec, double x, double y, int size) {
  double mx, my;
  mec_pos(a, mec, mx, my);
  const double dx = x - mx, dy = y - my;
  const double d = sqrt(dx * dx + dy * dy);
  const double pl_db = 128.1 + 37.6 * log10(d + 0.1);
  const double pl = pow(a.sp.path_loss, -pl_db / 10.0);
  const double rate = a.sp.bandwidth * log2(1.0 + (a.sp.cgl * a.sp.tx_power * pl) / a.sp.noise);
  const double tx = (double)size / rate * 1000.0;
  const double cmp = ((double)(a.sp.comp_cycles * size) / a.sp.mec_cap) * 1000.0;
  return round2_numpy(tx + cmp);
}

struct AgentView {
  int mec, len, size, thr, ack;
  double x, y;
};

__device__ __forceinline__ void load_agent(const EnvArgs& a, int e, int ag, AgentView& v) {
  const int i = e * a.A + ag;
  v.mec = a.s.mec_index[i];
  v.x = a.s.x[i];
  v.y = a.s.y[i];
  v.len = a.s.q_len[i];
  const int h = a.s.q_head[i];
  v.size = v.len ? a.s.q_size[(size_t)i * a.QMAX + h] : 0;
  v.thr = v.len ? a.s.q_thr[(size_t)i * a.QMAX + h] : 0;
  v.ack = a.s.last_ack[i];
}

// get_agent_inf (:123-146) -> inf[5]
__device__ __forceinline__ void agent_inf(const EnvArgs& a, const AgentView& v, double* inf) {
  if (v.len) {
    inf[0] = (double)v.size;
    inf[1] = rint(((double)(v.size * (int64_t)a.sp.comp_cycles) / a.sp.user_cap) * 1000.0);
    inf[2] = offload_delay(a, v.mec, v.x, v.y, v.size);
    inf[3] = (double)v.thr;
    inf[4] = (double)v.len;
  } else {
    inf[0] = inf[1] = inf[2] = inf[3] = inf[4] = 0.0;
  }
}

// ---- lane map: G envs per wave ---------------------------------------------
// A one-wave workgroup steps G = 64 / apad envs (apad = A rounded up to a power
// of two; fewer when the per-env collision counters would not fit the LDS):
// lane = g * apad + ag runs agent ag of env blockIdx.x * G + g in every per-agent
// phase, and the normaliser's G * len(obs) (env, feature) items are spread over
// all 64 lanes.  One env per wave left 48 of 64 lanes idle at 16 AGVs and, at
// 139 VGPRs (3 waves / SIMD), needed 8192 / 3072 -> three rounds of waves.
constexpr int FREQ_CAP = 1088;  // int counters: G * M * (C + 1)
constexpr int QR = 16;          // job queues up to this capacity are updated in registers

struct LaneMap {
  int apad, G;
};

__host__ inline LaneMap lane_map(int A, int M, int C) {
  int apad = 1;
  while (apad < A) apad *= 2;
  int G = 64 / apad;
  const int cap = FREQ_CAP / (M * (C + 1));
  return LaneMap{apad, G < cap ? G : cap};
}

// LDS scratch of one wave: per-agent arrays indexed by lane (g * apad + ag)
struct EnvLds {
  double inf[64][5];
  double dr[64];
  double rd[64];
  int mec[64];
  int ack[64];
  int tn[64], ts[64];
  int freq[FREQ_CAP];  // [g][mec][channel]
  int64_t n[64];       // [g] normaliser update count
};

struct Who {
  int lane, g, ag, e, gb;  // gb = g * apad: the group's first lane
  bool agent;              // lane runs an agent of a live env
  bool lead;               // lane is its live env's agent 0
};

__device__ __forceinline__ Who who(const EnvArgs& a) {
  Who w;
  w.lane = threadIdx.x & 63;
  w.g = w.lane / a.apad;
  w.ag = w.lane - w.g * a.apad;
  w.gb = w.g * a.apad;
  w.e = blockIdx.x * a.G + w.g;
  const bool live = w.g < a.G && w.e < a.NE;
  w.agent = live && w.ag < a.A;
  w.lead = live && w.ag == 0;
  return w;
}

// The env workgroups are one wave: an LDS read after other lanes' LDS writes needs
// program order only (a wave's LDS instructions complete in order), so the
// kernel's hand-overs between lanes are compiler fences.  __syncthreads() would
// also wait for every outstanding global load — at the step's first hand-over,
// the whole prefetched state.  (Global data is only ever re-read by the lane that
// wrote it.)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- compact observation wire format ---------------------
// Everything get_obs_agent (:148-182) reads about entity j, as 4 int32:
//   w0 size, w1 data_delay (get_agent_inf's round() to int), w2 the offload
//   delay in hundredths (the fp64 value is rint(x*100)/100, so rint(v*100) is
//   an exact integer k and k/100.0 reproduces v bit for bit),
//   w3 thr (bits 0-15) | queue length (16-23) | ack+1 (24-25) | mec_index (26-31).
// All fields are 0 when the queue is empty (get_agent_inf returns zeros).
// Together with the normaliser (n, mean, S) at the start of the episode, the
// wire records of t = 0..T reproduce every returned obs exactly (t2o_obs_expand).
__device__ __forceinline__ void write_wire(const EnvArgs& a, const Who& w, const EnvLds& L) {
  if (!a.o.wire || !w.agent) return;
  const double* inf = L.inf[w.lane];
  int4 v;
  v.x = (int)inf[0];
  v.y = (int)inf[1];
  v.z = (int)rint(inf[2] * 100.0);
  v.w = ((int)inf[3] & 0xFFFF) | ((int)inf[4] << 16) | ((L.ack[w.lane] + 1) << 24) | (L.mec[w.lane] << 26);
  reinterpret_cast<int4*>(a.o.wire)[(size_t)w.e * a.A + w.ag] = v;
}

// get_obs (:184-186) = A sequential normaliser updates per env; writes the obs if
// out, and the normaliser's (n, mean, S) at the end into the reset snapshot if
// snap.  Item q = lane + 64 k (k < OBS_SLOTS) is feature p = q % len of env
// g = q / len of the wave: its running (mean, S) live in registers over the A
// updates and reach HBM once at the end, with the last std (the only one read
// later).  Entity mode: feature p = 9 j + f of agent i's obs is entity j's field
// f if i and j share a MEC (f = 8: is_self), else 0 — j's value is fetched once
// per call, each update only compares i's MEC.  The IEEE operations and their
// order are the reference's.
constexpr int OBS_SLOTS = 9;  // ceil(G * 9A / 64) <= 9 for every A <= 64

// a / n correctly rounded from y = RN(1/n): q within 1.5 ulp, one correction
// brings it within one ulp, and Markstein's theorem makes the second exact (the
// remainders are exact fma results).  Preconditions, which the normaliser's
// operands meet: finite, far from the subnormal range, and never -0 (a = +0
// gives +0; x and the running mean are never -0, so neither is x - mean, and S
// is a sum of non-negative products from +0).  Checked against IEEE division on
// 5.9e7 random (a, n <= 3e5) pairs with gcc; tests/test_env_division.py keeps a
// 2e6-pair version of that check.
__device__ __forceinline__ double div_by(double a, double n, double y) {
  double q = a * y;
  double r = fma(-q, n, a);
  q = fma(r, y, q);
  r = fma(-q, n, a);
  return fma(r, y, q);
}

// sqrt(t) correctly rounded for t = +0 or t >= 2^-767: the f64 sqrt expansion the
// compiler emits (v_rsq_f64, then Goldschmidt / Newton steps on fma) without its
// range scaling, which only t < 2^-767 needs.  The normaliser's S / n is +0 or
// far above that: x lies on a grid of hundredths, so a non-zero running mean is
// >= 0.01 / n, every non-zero x - mean >= an ulp of that, and S is a sum of
// products of two such differences (>= 1e-68) over n < 2^53 updates.
__device__ __forceinline__ double sqrt_nn(double t) {
  const double r = __builtin_amdgcn_rsq(t);  // rsq(+0) = +inf
  double g = t * r, h = 0.5 * r;
  const double e = fma(-h, g, 0.5);
  g = fma(g, e, g);
  h = fma(h, e, h);
  double d = fma(-g, g, t);
  g = fma(d, h, g);
  d = fma(-g, g, t);
  g = fma(d, h, g);
  return t == 0.0 ? t : g;
}

// a / z correctly rounded for operands that need no range scaling: the f64
// division expansion the compiler emits (v_rcp_f64, two Newton steps on the
// reciprocal, one quotient correction) without v_div_scale / v_div_fmas /
// v_div_fixup, which only change the result for exponents near the ends of the
// range, zeros, infinities and NaNs.  Here z = std + 1e-8 in [1e-8, 1e7] and a =
// x - mean, |a| < 1e7, is +0 or >= 1e-34 (see sqrt_nn), so the results are the
// library's bit for bit.
__device__ __forceinline__ double div_lean(double a, double z) {
  double y = __builtin_amdgcn_rcp(z);
  double e = fma(-z, y, 1.0);
  y = fma(y, e, y);
  e = fma(-z, y, 1.0);
  y = fma(y, e, y);
  const double q = a * y;
  const double r = fma(-z, q, a);
  return fma(r, y, q);
}

// (q / d, q % d) for 0 <= q < 1024 and 1 <= d < 1024 through one fp32 multiply:
// (q + 1/2) / d keeps >= 1/(2d) >= 4.9e-4 from any integer, the product's error is
// below 1024 * 2^-23 = 1.2e-4 (rd = RN(1/d)).  Replaces a runtime integer division.
__device__ __forceinline__ void divmod_small(int q, int d, float rd, int& g, int& p) {
  g = (int)(((float)q + 0.5f) * rd);
  p = q - g * d;
}

// The fast normaliser loop of get_obs (every env of the wave at the same count
// n0 >= 1, so each update divides by the wave-uniform n >= 2: one reciprocal per
// update and Markstein's correction, div_by, instead of one IEEE division per
// item).  Entity mode: x = xv if agent i's MEC equals key (j's MEC), or, for the
// is_self feature (key = -1 - j), if i == j; else 0.  Flat mode: x is agent i's
// own feature p.  The obs go through range-checked buffers over this wave's envs:
// an item past the last env / feature has an out-of-range offset, so it is
// computed (on lane data of group 0) and dropped.
template <bool OUT, bool ENT>
__device__ __attribute__((always_inline)) void norm_fast(const EnvArgs& a, const Who& w, const EnvLds& L, int64_t nref,
                                                        double (&mr)[OBS_SLOTS], double (&sr)[OBS_SLOTS],
                                                        const double (&xv)[OBS_SLOTS], const int (&key)[OBS_SLOTS],
                                                        const int (&gq)[OBS_SLOTS]) {
  const int A = a.A, no = obs_len(ENT, A);
  const int e0 = blockIdx.x * a.G, ne = a.NE - e0 < a.G ? a.NE - e0 : a.G;
  float* obase = a.o.obs ? a.o.obs + (size_t)e0 * A * no : nullptr;
  double* obase64 = a.o.obs64 ? a.o.obs64 + (size_t)e0 * A * no : nullptr;
  const __amdgpu_buffer_rsrc_t orsrc =
      __builtin_amdgcn_make_buffer_rsrc(obase, (short)0, a.o.obs ? ne * A * no * (int)sizeof(float) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t orsrc64 = __builtin_amdgcn_make_buffer_rsrc(
      obase64, (short)0, a.o.obs64 ? ne * A * no * (int)sizeof(double) : 0, 0x00020000);
  const float rno = 1.0f / (float)no;
  int ooff[OBS_SLOTS];  // bytes into the float obs; 2 * ooff (unsigned) into the fp64 copy
  int lb[OBS_SLOTS];    // LDS lane of agent 0 of the item's env
#pragma unroll
  for (int k = 0; k < OBS_SLOTS; ++k) {
    int g, p;
    divmod_small(w.lane + 64 * k, no, rno, g, p);
    ooff[k] = gq[k] < 0 ? 0x40000000 : (g * A * no + p) * (int)sizeof(float);
    lb[k] = gq[k] < 0 ? 0 : gq[k];
  }
  const double n0 = (double)nref;
  for (int i = 0; i < A; ++i) {
    const double n = n0 + (double)(i + 1);
    const double y = 1.0 / n;
    const int self = -1 - i;
#pragma unroll
    for (int k = 0; k < OBS_SLOTS; ++k) {
      double x;
      if constexpr (ENT) {
        const int mi = L.mec[lb[k] + i];
        x = (mi == key[k] || self == key[k]) ? xv[k] : 0.0;
      } else {
        int g, p;
        divmod_small(w.lane + 64 * k, no, rno, g, p);
        x = p == 0 ? (double)L.ack[lb[k] + i] : L.inf[lb[k] + i][p - 1];  // [last_ack (raw -1/0/1), get_agent_inf]
      }
      const double old = mr[k], dx = x - old;
      const double m = old + div_by(dx, n, y);
      const double sn = sr[k] + dx * (x - m);
      mr[k] = m;
      sr[k] = sn;
      if constexpr (OUT) {
        const double v = div_lean(x - m, sqrt_nn(div_by(sn, n, y)) + 1e-8);
        if (a.o.obs)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, (float)v), orsrc, ooff[k],
                                                i * no * (int)sizeof(float), 0);
        if (a.o.obs64) {
          typedef int v2i __attribute__((ext_vector_type(2)));
          // (doubled in unsigned arithmetic: the drop sentinel 0x40000000 becomes
          // 0x80000000, still past the range-checked buffer's end)
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, v), orsrc64,
                                                __builtin_bit_cast(int, (unsigned)ooff[k] << 1),
                                                i * no * (int)sizeof(double), 0);
        }
      }
    }
  }
}

// This lane's normaliser items (mean, S), loaded once per launch (in step mode at
// the kernel's start, so the loads overlap the step) and carried across get_obs
// calls in registers.
struct NormPre {
  double mr[OBS_SLOTS], sr[OBS_SLOTS];
};

__device__ __forceinline__ void load_norm(const EnvArgs& a, const Who& w, NormPre& pre) {
  const int A = a.A, n9 = 9 * A, no = obs_len(a.sp.obs_entity, A), items = a.G * no;
  const float rno = 1.0f / (float)no;
#pragma unroll
  for (int k = 0; k < OBS_SLOTS; ++k) {
    const int q = w.lane + 64 * k;
    int g, p;
    divmod_small(q, no, rno, g, p);
    const int e = blockIdx.x * a.G + g;
    pre.mr[k] = pre.sr[k] = 0.0;
    if (q < items && e < a.NE) {
      pre.mr[k] = a.s.nrm_mean[(size_t)e * n9 + p];
      pre.sr[k] = a.s.nrm_S[(size_t)e * n9 + p];
    }
  }
}

template <bool OUT>
__device__ __attribute__((always_inline)) void get_obs(const EnvArgs& a, const Who& w, EnvLds& L, NormPre& pre,
                                                      bool snap) {
  // normaliser rows keep their [9A] stride in both modes (state[14..16])
  const int A = a.A, n9 = 9 * A, no = obs_len(a.sp.obs_entity, A);
  const int items = a.G * no;
  const float rno = 1.0f / (float)no;
  double(&mr)[OBS_SLOTS] = pre.mr;
  double(&sr)[OBS_SLOTS] = pre.sr;
  double xv[OBS_SLOTS];
  int64_t n0[OBS_SLOTS];  // the env's update count before this call
  int key[OBS_SLOTS];  // entity mode: j's MEC, or -1 - j for is_self
  int gq[OBS_SLOTS];   // the item's group base lane (-1: no item)
#pragma unroll
  for (int k = 0; k < OBS_SLOTS; ++k) {
    const int q = w.lane + 64 * k;
    int g, p;
    divmod_small(q, no, rno, g, p);
    const int e = blockIdx.x * a.G + g;
    gq[k] = -1;
    xv[k] = 0.0;
    key[k] = n0[k] = 0;
    if (q < items && e < a.NE) {
      gq[k] = g * a.apad;
      n0[k] = L.n[g];
      if (a.sp.obs_entity) {
        const int j = p / 9, f = p - 9 * (p / 9), lj = gq[k] + j;
        if (f < 3) xv[k] = (f == L.ack[lj] + 1) ? 1.0 : 0.0;  // ack_mapping: -1 -> [1,0,0], 0 -> [0,1,0], 1 -> [0,0,1]
        else if (f < 8) xv[k] = L.inf[lj][f - 3];
        else xv[k] = 1.0;
        key[k] = f == 8 ? -1 - j : L.mec[lj];
      }
    }
  }
  // every env of the wave at the same update count n0 >= 1: always, past the first
  // reset's first call
  const int64_t nref = L.n[0];
  bool same = true;
#pragma unroll
  for (int k = 0; k < OBS_SLOTS; ++k) same = same && (gq[k] < 0 || n0[k] == nref);
  if (__all(same) && nref >= 1) {
    if (a.sp.obs_entity) norm_fast<OUT, true>(a, w, L, nref, mr, sr, xv, key, gq);
    else norm_fast<OUT, false>(a, w, L, nref, mr, sr, xv, key, gq);
  } else {
    for (int i = 0; i < A; ++i) {
  #pragma unroll
      for (int k = 0; k < OBS_SLOTS; ++k) {
        if (gq[k] < 0) continue;
        int g, p;
        divmod_small(w.lane + 64 * k, no, rno, g, p);
        const int li = gq[k] + i;
        double x;
        if (a.sp.obs_entity) {
          x = (L.mec[li] == key[k] || -1 - i == key[k]) ? xv[k] : 0.0;
        } else {
          x = p == 0 ? (double)L.ack[li] : L.inf[li][p - 1];  // [last_ack (raw -1/0/1), get_agent_inf]
        }
        const double n = (double)(n0[k] + i + 1);
        double m, s;
        if (n == 1.0) {
          m = x;
          s = sr[k];
        } else {
          const double old = mr[k];
          m = old + (x - old) / n;
          s = sr[k] + (x - old) * (x - m);
        }
        mr[k] = m;
        sr[k] = s;
        if (OUT) {
          const double d = n == 1.0 ? x : sqrt(s / n);
          const double v = (x - m) / (d + 1e-8);
          const size_t o = ((size_t)(blockIdx.x * a.G + g) * A + i) * no + p;
          if (a.o.obs) a.o.obs[o] = (float)v;
          if (a.o.obs64) a.o.obs64[o] = v;
        }
      }
    }
  }
  // (validity and counts re-derived here, so the per-item arrays above need not
  // stay live through the update loop)
#pragma unroll
  for (int k = 0; k < OBS_SLOTS; ++k) {
    const int q = w.lane + 64 * k;
    int g, p;
    divmod_small(q, no, rno, g, p);
    const int e = blockIdx.x * a.G + g;
    if (q >= items || e >= a.NE) continue;
    const size_t r = (size_t)e * n9 + p;
    const double n = (double)(L.n[g] + A);
    a.s.nrm_mean[r] = mr[k];
    a.s.nrm_S[r] = sr[k];
    a.s.nrm_std[r] = n == 1.0 ? mr[k] : sqrt(sr[k] / n);  // the last update's std (at n = 1: x = mean)
    if (snap) {  // the normaliser the episode's first returned obs starts from
      a.o.snap[(size_t)e * 2 * n9 + p] = mr[k];
      a.o.snap[(size_t)e * 2 * n9 + n9 + p] = sr[k];
    }
  }
  wave_sync();  // every item read L.n before the count moves on
  if (w.lead) {
    L.n[w.g] += A;
    if (snap) a.o.snap_n[w.e] = L.n[w.g];
  }
  wave_sync();
}

__device__ __forceinline__ void fill_lds(const EnvArgs& a, const Who& w, EnvLds& L) {
  if (w.agent) {
    AgentView v;
    load_agent(a, w.e, w.ag, v);
    L.mec[w.lane] = v.mec;
    L.ack[w.lane] = v.ack;
    agent_inf(a, v, L.inf[w.lane]);
  }
  wave_sync();
}

__device__ __forceinline__ void write_state_avail(const EnvArgs& a, const Who& w, const EnvLds& L) {
  const int A = a.A, nA = a.C + 1, ns = 8 * A;
  if (a.o.state) {
    for (int g = 0; g < a.G; ++g) {
      const int e = blockIdx.x * a.G + g;
      if (e >= a.NE) break;
      const int gb = g * a.apad;
      for (int p = w.lane; p < ns; p += 64) {
        float v;
        if (p < 3 * A) {
          const int j = p / 3, f = p % 3;
          v = (f == L.ack[gb + j] + 1) ? 1.f : 0.f;
        } else {
          const int r = p - 3 * A;
          v = (float)L.inf[gb + r / 5][r % 5];
        }
        a.o.state[(size_t)e * ns + p] = v;
      }
    }
  }
  if (a.o.avail && w.agent) {
    const bool has = L.inf[w.lane][4] > 0.0;  // get_agent_inf's queue length
    for (int k = 0; k < nA; ++k)
      a.o.avail[((size_t)w.e * A + w.ag) * nA + k] = has ? (a.sp.edge_only ? k != 0 : 1) : k == 0;
  }
}

// appends a job with probability arrival_p to the queue (head, len); returns its
// size, 0 if none arrived (sizes are >= size_min >= 1)
__device__ __forceinline__ int generate_job(const EnvArgs& a, int i, int head, int len, double u1, double u2) {
  if (u1 < a.sp.arrival_p) {
    const int slot = (head + len) % a.QMAX;
    const int size = a.sp.size_min + (int)(u2 * (double)(a.sp.size_max - a.sp.size_min + 1));
    a.s.q_size[(size_t)i * a.QMAX + slot] = size;
    a.s.q_thr[(size_t)i * a.QMAX + slot] = a.sp.latency_max;
    a.s.q_len[i] = len + 1;
    a.s.task_num[i] += 1;
    return size;
  }
  return 0;
}

// One step (:309-366) of the wave's envs.  Every per-agent state the step reads
// — position, MEC, job queue (thresholds and sizes, in registers when the queue
// capacity is <= QR), counters, the action — is loaded up front in one batch, the
// normaliser items after them, so the step pays about one memory round trip;
// everything after computes from registers and only stores.
__device__ __forceinline__ void env_step(const EnvArgs& a, const Who& w, EnvLds& L, NormPre& pre) {
  const int A = a.A, M = a.M, C = a.C, FS = M * (C + 1), Q = a.QMAX;
  const bool ring = Q <= QR;
  const int i = w.e * A + w.ag;
  int mec = 0, len = 0, head = 0, act = 0, tnum = 0, tsucc = 0;
  double x = 0.0, y = 0.0, rdel = 0.0;
  int thr[QR], size[QR];
#pragma unroll
  for (int k = 0; k < QR; ++k) thr[k] = size[k] = 0;
  int* thr_ring = a.s.q_thr + (size_t)i * Q;
  int* size_ring = a.s.q_size + (size_t)i * Q;
  if (w.agent) {
    mec = a.s.mec_index[i];
    x = a.s.x[i];
    y = a.s.y[i];
    len = a.s.q_len[i];
    head = a.s.q_head[i];
    act = (int)a.actions[(int64_t)w.e * a.act_se + w.ag];
    tnum = a.s.task_num[i];
    tsucc = a.s.task_success[i];
    rdel = a.s.remain_delay[i];
    if (ring) {
#pragma unroll
      for (int k = 0; k < QR; ++k)
        if (k < Q) {
          thr[k] = thr_ring[k];
          size[k] = size_ring[k];
        }
    }
  }
  int64_t base = 0, nrm = 0;
  int tslot = 0;
  if (w.agent) base = a.s.draw[w.e];
  if (w.lead) {
    nrm = a.s.nrm_n[w.e];
    tslot = a.s.time_slot[w.e];
  }
  load_norm(a, w, pre);
  for (int k = w.lane; k < a.G * FS; k += 64) L.freq[k] = 0;
  if (w.lead) L.n[w.g] = nrm;
  wave_sync();
  // the head job (load_agent)
  int hsize = 0, hthr = 0;
  if (w.agent && len) {
    if (ring) {
#pragma unroll
      for (int k = 0; k < QR; ++k) {
        hsize = k == head ? size[k] : hsize;
        hthr = k == head ? thr[k] : hthr;
      }
    } else {
      hsize = size_ring[head];
      hthr = thr_ring[head];
    }
  }
  int* freq = L.freq + w.g * FS;
  if (w.agent) {
    act = act < 0 ? 0 : (act > C ? C : act);  // actions come from avail-masked selection; clamp keeps LDS in bounds
    atomicAdd(&freq[mec * (C + 1) + act], 1);
  }
  wave_sync();
  int ack = 0;
  if (w.agent) {
    if (act == 0) ack = 0;
    else ack = (freq[mec * (C + 1) + act] == 1) ? 1 : -1;
  }
  // get_reward (:229-293): per-agent terms, summed in agent order below
  double dr = 0.0, rd_inc = 0.0;
  int over = 0, succ = 0;
  bool has_dr = false;
  if (w.agent && len) {
    const double local = round2_python(((double)(a.sp.comp_cycles * hsize) / a.sp.user_cap) * 1000.0);
    if (ack == 0) {
      if ((double)hthr - local > 0) {
        succ = 1;
        rd_inc = (double)(a.sp.latency_max - hthr) + local;
      } else {
        over = a.sp.latency_max;
      }
    } else if (ack == -1) {
      if (hthr - a.sp.t_length <= 0) over = a.sp.latency_max;
    } else {
      const double off = offload_delay(a, mec, x, y, hsize);
      dr = local - off;
      has_dr = true;
      if ((double)hthr - off > 0) {
        succ = 1;
        rd_inc = (double)(a.sp.latency_max - hthr) + off;
      } else {
        over = a.sp.latency_max;
      }
    }
  }
  if (w.agent) {
    L.dr[w.lane] = has_dr ? dr : NAN;
    L.ack[w.lane] = ack;
    L.mec[w.lane] = mec;
    L.tn[w.lane] = over;
  }
  wave_sync();
  if (w.lead) {
    // channel utilisation (:321-329): counts > 1 zeroed, Python sums in order; a
    // kept count is 0 or 1, so each term is +0 or the one quotient 1 / C
    const double inv_c = 1.0 / (double)C;
    double util = 0.0;
    for (int m = 0; m < M; ++m) {
      double su = 0.0;
      for (int c = 0; c <= C; ++c) su = su + (freq[m * (C + 1) + c] == 1 ? inv_c : 0.0);
      util = util + su;
    }
    util = util / (double)M;
    double delay_reward = 0.0;
    int overtime = 0, confl = 0;
    for (int ag = 0; ag < A; ++ag) {
      if (!isnan(L.dr[w.gb + ag])) delay_reward = delay_reward + L.dr[w.gb + ag];
      overtime += L.tn[w.gb + ag];
      confl += L.ack[w.gb + ag] == -1;
    }
    a.o.reward[w.e] = delay_reward - (double)overtime;
    double* info = a.o.info + (size_t)w.e * 6;
    info[0] = delay_reward;
    info[1] = (double)overtime;
    info[2] = util;
    info[3] = (double)confl / (double)A;
    info[4] = info[5] = NAN;
  }
  wave_sync();
  // update_users (:295-307) after the reward, agent by agent (independent)
  AgentView nv{};
  if (w.agent) {
    a.s.last_ack[i] = ack;
    if (a.o.ack) a.o.ack[i] = ack;
    tsucc += succ;
    a.s.task_success[i] = tsucc;
    rdel = rdel + rd_inc;
    a.s.remain_delay[i] = rdel;
    const int64_t b = base + 5 * w.ag;
    const int m = (int)(uniform(a.seed, w.e, b) * (double)M);  // only places the AGV: mec_index stays
    double px, py;
    position(a, m, uniform(a.seed, w.e, b + 1), uniform(a.seed, w.e, b + 2), px, py);
    a.s.x[i] = px;
    a.s.y[i] = py;
    if (ack != -1 && len > 0) {
      head = (head + 1) % Q;
      --len;
    }
    // every queued job's threshold drops by t_length (5); the expired ones are a
    // FIFO prefix (thresholds grow from head to tail: jobs arrive with latency_max
    // and age together), so they are counted, not searched
    if (ring) {
      int nexp = 0;
#pragma unroll
      for (int k = 0; k < QR; ++k) {
        int rel = k - head;
        rel = rel < 0 ? rel + Q : rel;
        if (k < Q && rel < len) {
          thr[k] -= 5;
          thr_ring[k] = thr[k];
          nexp += thr[k] <= 0;
        }
      }
      head = (head + nexp) % Q;
      len -= nexp;
    } else {
      for (int k = 0; k < len; ++k) thr_ring[(head + k) % Q] -= 5;
      while (len > 0 && thr_ring[head] <= 0) {
        head = (head + 1) % Q;
        --len;
      }
    }
    a.s.q_head[i] = head;
    a.s.q_len[i] = len;
    const int nsize = generate_job(a, i, head, len, uniform(a.seed, w.e, b + 3), uniform(a.seed, w.e, b + 4));
    tnum += nsize > 0;
    // the new state as get_agent_inf sees it (load_agent without re-reading it)
    int nh_size = nsize, nh_thr = nsize > 0 ? a.sp.latency_max : 0;
    if (len > 0) {
      if (ring) {
#pragma unroll
        for (int k = 0; k < QR; ++k) {
          nh_size = k == head ? size[k] : nh_size;
          nh_thr = k == head ? thr[k] : nh_thr;
        }
      } else {
        nh_size = size_ring[head];
        nh_thr = thr_ring[head];
      }
    }
    nv.mec = mec;
    nv.x = px;
    nv.y = py;
    nv.ack = ack;
    nv.len = len + (nsize > 0);
    nv.size = nh_size;
    nv.thr = nh_thr;
    L.tn[w.lane] = tnum;
    L.ts[w.lane] = tsucc;
    L.rd[w.lane] = rdel;
  }
  wave_sync();
  if (w.lead) {
    a.s.draw[w.e] = base + 5 * A;
    const int ts = tslot + 1;
    a.s.time_slot[w.e] = ts;
    const bool term = ts == a.T;
    a.o.terminated[w.e] = term ? 1 : 0;
    if (term) {  // get_task_num (:368-415)
      int tn = 0, tsu = 0;
      double rd = 0.0;
      for (int ag = 0; ag < A; ++ag) {
        tn += L.tn[w.gb + ag];
        tsu += L.ts[w.gb + ag];
        rd = rd + L.rd[w.gb + ag];
      }
      double* info = a.o.info + (size_t)w.e * 6;
      info[4] = (double)tsu / (double)tn;
      info[5] = tsu != 0 ? rd / (double)tsu : 0.0;
    }
  }
  // the worker's get_state / get_avail_actions / get_obs on the new state
  if (w.agent) {
    L.mec[w.lane] = nv.mec;
    L.ack[w.lane] = nv.ack;
    agent_inf(a, nv, L.inf[w.lane]);
  }
  wave_sync();
  write_state_avail(a, w, L);
  write_wire(a, w, L);
  get_obs<true>(a, w, L, pre, false);
  if (w.lead) a.s.nrm_n[w.e] = L.n[w.g];
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void env_kernel(EnvArgs a) {
  __shared__ EnvLds L;
  const Who w = who(a);
  const int A = a.A, M = a.M;
  if (blockIdx.x * a.G >= a.NE) return;
  const bool live = w.g < a.G && w.e < a.NE;
  const int64_t base = a.mode == 0 || a.mode == 2 || !live ? 0 : a.s.draw[w.e];
  if (a.mode == 0) {  // construction (:25-40): mec_index + position per agent
    if (w.agent) {
      const int i = w.e * A + w.ag;
      const double u0 = uniform(a.seed, w.e, base + 3 * w.ag), u1 = uniform(a.seed, w.e, base + 3 * w.ag + 1),
                   u2 = uniform(a.seed, w.e, base + 3 * w.ag + 2);
      const int m = (int)(u0 * (double)M);
      a.s.mec_index[i] = m;
      position(a, m, u1, u2, a.s.x[i], a.s.y[i]);
      a.s.q_head[i] = a.s.q_len[i] = 0;
      a.s.task_num[i] = a.s.task_success[i] = 0;
      a.s.remain_delay[i] = 0.0;
      a.s.last_ack[i] = 0;
    }
    const int n9 = 9 * A;
    for (int q = w.lane; q < a.G * n9; q += 64) {
      const int e = blockIdx.x * a.G + q / n9;
      if (e >= a.NE) break;
      const size_t r = (size_t)e * n9 + q % n9;
      a.s.nrm_mean[r] = a.s.nrm_S[r] = a.s.nrm_std[r] = 0.0;
    }
    if (w.lead) {
      a.s.nrm_n[w.e] = 0;
      a.s.time_slot[w.e] = 0;
      a.s.draw[w.e] = base + 3 * A;
    }
    return;
  }
  if (w.lead && a.mode != 2) L.n[w.g] = a.s.nrm_n[w.e];
  NormPre pre;
  if (a.mode == 3) {  // get_env_info (:421-439): two get_obs calls (one without entity obs, :425,431-434)
    load_norm(a, w, pre);
    fill_lds(a, w, L);
    get_obs<false>(a, w, L, pre, false);
    if (a.sp.obs_entity) get_obs<false>(a, w, L, pre, false);
    if (w.lead) a.s.nrm_n[w.e] = L.n[w.g];
    return;
  }
  if (a.mode == 1) {  // reset (:219-227), then the worker's get_state/get_avail/get_obs
    if (w.agent) {
      const int i = w.e * A + w.ag;
      const int64_t b = base + 5 * w.ag;
      const int m = (int)(uniform(a.seed, w.e, b) * (double)M);
      position(a, m, uniform(a.seed, w.e, b + 1), uniform(a.seed, w.e, b + 2), a.s.x[i], a.s.y[i]);
      a.s.q_head[i] = a.s.q_len[i] = 0;
      a.s.task_num[i] = a.s.task_success[i] = 0;
      a.s.remain_delay[i] = 0.0;
      generate_job(a, i, 0, 0, uniform(a.seed, w.e, b + 3), uniform(a.seed, w.e, b + 4));
      a.s.last_ack[i] = 0;
    }
    if (w.lead) {
      a.s.time_slot[w.e] = 0;
      a.s.draw[w.e] = base + 5 * A;
    }
    wave_sync();
    load_norm(a, w, pre);
    fill_lds(a, w, L);
    get_obs<false>(a, w, L, pre, a.o.snap != nullptr);  // reset()'s own get_obs
    write_state_avail(a, w, L);
    write_wire(a, w, L);
    get_obs<true>(a, w, L, pre, false);  // the worker's get_obs
    if (w.lead) a.s.nrm_n[w.e] = L.n[w.g];
    return;
  }
  // ---- step (:309-366)
  env_step(a, w, L, pre);
}

// ---- t2o_obs_expand: wire records -> dense normalised obs --------------------
// One thread per (episode b, feature p = 9j + f), flattened over b·9A so every
// CU gets waves whatever A is: the normaliser is elementwise, so feature p's
// running (mean, S) is a private chain over (t, agent i) in the reference's order
// (get_obs updates agent by agent, normalization.py:12-35), with the same IEEE
// operations as get_obs above.  Each one-wave workgroup stages the wire rows of
// the (at most A·(64/9A + 2) <= 128) episode rows its lanes touch at step t in
// LDS and reads them as broadcasts.  The chain is fp64 division/sqrt bound.
constexpr int XP_THREADS = 64;
constexpr int XP_ROWS = 128;

struct ExpandArgs {
  const int32_t* wire;
  int64_t w_sb, w_st;  // int32-element strides of episode / step
  const int64_t* snap_n;
  const double* snap;  // [B][2][9A]
  float* obs;
  int64_t o_sb, o_st;  // float-element strides of episode / step
  double* obs64;       // dense [B][T1][A][9A] or null
  int B, T1, A;
};

__global__ __launch_bounds__(XP_THREADS) void obs_expand_kernel(ExpandArgs a) {
  __shared__ int4 rows[XP_ROWS];  // [(episode - b0) * A + agent]
  const int A = a.A, n9 = 9 * A;
  const int64_t total = (int64_t)a.B * n9;
  const int64_t g0 = (int64_t)blockIdx.x * XP_THREADS;
  const int64_t gid = g0 + threadIdx.x;
  const bool live = gid < total;
  const int b0 = (int)(g0 / n9);
  const int b1 = (int)(((g0 + XP_THREADS < total ? g0 + XP_THREADS : total) - 1) / n9);
  const int nrows = (b1 - b0 + 1) * A;
  const int b = live ? (int)(gid / n9) : b0;
  const int p = (int)(gid - (int64_t)b * n9);
  const int j = p / 9, f = p % 9;
  const int rb = (b - b0) * A;
  double mean = 0.0, S = 0.0;
  int64_t n = 0;
  if (live) {
    n = a.snap_n[b];
    mean = a.snap[(size_t)b * 2 * n9 + p];
    S = a.snap[(size_t)b * 2 * n9 + n9 + p];
  }
  for (int t = 0; t < a.T1; ++t) {
    __syncthreads();
    for (int r = threadIdx.x; r < nrows; r += XP_THREADS)
      rows[r] = *reinterpret_cast<const int4*>(a.wire + (size_t)(b0 + r / A) * a.w_sb + (size_t)t * a.w_st +
                                               4 * (r % A));
    __syncthreads();
    if (!live) continue;
    const int4 wj = rows[rb + j];
    const int mec_j = (wj.w >> 26) & 63;
    double xj;  // entity j's field f as seen from an agent of the same MEC (f < 8)
    switch (f) {
      case 0: case 1: case 2: xj = (f == ((wj.w >> 24) & 3)) ? 1.0 : 0.0; break;
      case 3: xj = (double)wj.x; break;
      case 4: xj = (double)wj.y; break;
      case 5: xj = (double)wj.z / 100.0; break;
      case 6: xj = (double)(wj.w & 0xFFFF); break;
      default: xj = (double)((wj.w >> 16) & 0xFF); break;
    }
    float* orow = a.obs ? a.obs + (size_t)b * a.o_sb + (size_t)t * a.o_st : nullptr;
    double* orow64 = a.obs64 ? a.obs64 + (((size_t)b * a.T1 + t) * A) * n9 : nullptr;
    for (int i = 0; i < A; ++i) {
      ++n;
      const int mec_i = (rows[rb + i].w >> 26) & 63;
      double x = 0.0;
      if (mec_i == mec_j) x = f < 8 ? xj : (i == j ? 1.0 : 0.0);
      double m, v;
      if (n == 1) {
        m = x;
        v = (x - m) / (x + 1e-8);
      } else {
        const double old = mean;
        m = old + (x - old) / (double)n;
        S = S + (x - old) * (x - m);
        v = (x - m) / (sqrt(S / (double)n) + 1e-8);
      }
      mean = m;
      if (orow) orow[(size_t)i * n9 + p] = (float)v;
      if (orow64) orow64[(size_t)i * n9 + p] = v;
    }
  }
}
}  // namespace

extern "C" int t2o_env_run_ex(int mode, const double* spec, void* const* state, void* const* out, int n_out,
                              const int64_t* actions, int64_t act_se, int NE, int A, int M, int C, int QMAX, int T,
                              uint64_t seed, void* stream) {
  if ((out && n_out != 8 && n_out != 11) || (n_out == 11 && out && (out[9] == nullptr) != (out[10] == nullptr)) ||
      (spec && (int)spec[9] > 0xFFFF) || QMAX > 255 ||
      (spec && spec[15] == 0.0 && n_out == 11 && out && (out[8] || out[9])))  // wire format: entity obs only
    return T2O_EINVAL;
  if (NE < 1 || A < 1 || A > MAXA || M < 1 || M > 16 || C < 1 || C > 16 || QMAX < 1 || !spec || !state ||
      (mode == 2 && (!actions || !out)) || (mode == 1 && !out) || mode < 0 || mode > 3)
    return T2O_EINVAL;
  EnvArgs a{};
  a.sp = EnvSpec{spec[0], spec[1], spec[2], spec[3], spec[4], spec[5], spec[6], spec[7], spec[8],
                 (int)spec[9], (int)spec[10], (int)spec[11], (int)spec[12], spec[13], spec[14] != 0.0,
                 spec[15] != 0.0};
  a.s = EnvState{(int32_t*)state[0], (double*)state[1], (double*)state[2], (int32_t*)state[3],
                 (int32_t*)state[4], (int32_t*)state[5], (int32_t*)state[6], (int32_t*)state[7],
                 (int32_t*)state[8], (double*)state[9], (int32_t*)state[10], (int32_t*)state[11],
                 (int64_t*)state[12], (int64_t*)state[13], (double*)state[14], (double*)state[15],
                 (double*)state[16]};
  if (out)
    a.o = EnvOut{(float*)out[0], (double*)out[1], (float*)out[2], (int32_t*)out[3], (double*)out[4],
                 (uint8_t*)out[5], (double*)out[6], (int32_t*)out[7], nullptr, nullptr, nullptr};
  if (out && n_out == 11) {
    a.o.wire = (int32_t*)out[8];
    a.o.snap_n = (int64_t*)out[9];
    a.o.snap = (double*)out[10];
  }
  a.actions = actions;
  a.act_se = act_se;
  a.NE = NE;
  a.A = A;
  a.M = M;
  a.C = C;
  a.QMAX = QMAX;
  a.T = T;
  a.seed = seed;
  a.mode = mode;
  const LaneMap lm = lane_map(A, M, C);
  a.apad = lm.apad;
  a.G = lm.G;
  hipLaunchKernelGGL(env_kernel, dim3((NE + lm.G - 1) / lm.G), dim3(64), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

extern "C" int t2o_env_run(int mode, const double* spec, void* const* state, void* const* out,
                           const int64_t* actions, int64_t act_se, int NE, int A, int M, int C, int QMAX, int T,
                           uint64_t seed, void* stream) {
  if (!spec) return T2O_EINVAL;
  double sp16[16];
  for (int i = 0; i < 15; ++i) sp16[i] = spec[i];
  sp16[15] = 1.0;  // entity observations
  return t2o_env_run_ex(mode, sp16, state, out, 8, actions, act_se, NE, A, M, C, QMAX, T, seed, stream);
}

extern "C" int t2o_obs_expand(const int32_t* wire, int64_t w_sb, int64_t w_st, const int64_t* snap_n,
                              const double* snap, float* obs, int64_t o_sb, int64_t o_st, double* obs64, int B,
                              int T1, int A, void* stream) {
  if (!wire || !snap_n || !snap || (!obs && !obs64) || B < 1 || T1 < 1 || A < 1 || A > MAXA ||
      (w_sb | w_st) % 4 != 0 || (obs && o_st < (int64_t)A * 9 * A) || (obs && B > 1 && o_sb < (int64_t)A * 9 * A))
    return T2O_EINVAL;
  if (((uintptr_t)wire & 15) != 0) return T2O_EINVAL;
  ExpandArgs a{wire, w_sb, w_st, snap_n, snap, obs, o_sb, o_st, obs64, B, T1, A};
  const int64_t blocks = ((int64_t)B * 9 * A + XP_THREADS - 1) / XP_THREADS;
  hipLaunchKernelGGL(obs_expand_kernel, dim3((unsigned)blocks), dim3(XP_THREADS), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
