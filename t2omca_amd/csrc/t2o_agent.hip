// t2o_agent.hip — TransformerAgent unrolled over a replay batch on MI355X.
//
// Reference: transf_agent.py:54-76 (+ transformer.py:40-178), called once per
// timestep by the MAC for t = 0..T of every sampled episode.  Here ONE launch
// runs the whole unroll: the agent is recurrent only through h, and every
// (episode, agent) sequence is independent, so a wave owns 16 sequences and
// carries their hidden state in registers across all timesteps (no inter-
// workgroup synchronisation at all).  A second network (the target agent) can
// run in the same launch on the same observations (blockIdx.y).
#include "t2o_agent_block.hpp"
#include "t2o_dispatch.hpp"

using namespace t2o;

namespace {

struct AgentNet {
  const float* pack;
  const float* h0;
  float* q;
  float* h;
};

struct AgentFwdArgs {
  t2o_layout L;
  AgentNet net[2];
  const float* obs;
  int64_t obs_sb, obs_st;
  int B, T, A, F;
};

template <int E, int H, int D, int NE, int FF>
__global__ __launch_bounds__(256) void agent_fwd_kernel(AgentFwdArgs args) {
  constexpr int ET = E / 16;
  const AgentNet net = args.net[blockIdx.y];
  const t2o_layout& L = args.L;
  const int A = args.A, F = args.F;
  const int R = args.B * A;
  const int rt = blockIdx.x * 4 + wave_id();
  if (rt * 16 >= R) return;  // wave-uniform: this kernel has no barriers
  const int c = lane_c(), g = lane_g();
  const int row_raw = rt * 16 + c;
  const bool valid = row_raw < R;
  const int row = valid ? row_raw : R - 1;
  const int b = row / A, a = row % A;
  const float* __restrict__ P = net.pack;

  f4 h[ET];
#pragma unroll
  for (int t = 0; t < ET; ++t) h[t] = net.h0 ? ld4(net.h0 + (size_t)row * E + 16 * t + 4 * g) : zero4();

  for (int step = 0; step < args.T; ++step) {
    const float* ob = args.obs + b * args.obs_sb + step * args.obs_st + (int64_t)a * NE * F;
    f4 o[NE];
#pragma unroll
    for (int j = 0; j < NE; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 4 * g + r;
        o[j][r] = f < F ? ob[j * F + f] : 0.f;
      }
    f4 x[ET];
#pragma unroll
    for (int t = 0; t < ET; ++t) x[t] = h[t];
#pragma unroll
    for (int d = 0; d < D; ++d) agent_block_fwd<E, H, NE, FF, false>(P, L, d, h, o, x, nullptr);
    f4 q = zero4();
#pragma unroll
    for (int i = 0; i < ET; ++i) q = mma_tile(P + L.Wo, E, 0, i, x[i], q);
    q += vec_t(P + L.bo, 0);
#pragma unroll
    for (int t = 0; t < ET; ++t) h[t] = x[t];
    if (valid) {
      const size_t base = ((size_t)b * args.T + step) * A + a;
      float* qo = net.q + base * L.NA;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r < L.NA) qo[4 * g + r] = q[r];
      float* ho = net.h + base * E;
#pragma unroll
      for (int t = 0; t < ET; ++t) st4(ho + 16 * t + 4 * g, h[t]);
    }
  }
}

template <int E, int H, int D, int NE, int FF>
int launch_fwd(const AgentFwdArgs& args, int nnet, hipStream_t stream) {
  const int R = args.B * args.A;
  const int tiles = (R + 15) / 16;
  dim3 grid((tiles + 3) / 4, nnet);
  hipLaunchKernelGGL((agent_fwd_kernel<E, H, D, NE, FF>), grid, dim3(256), 0, stream, args);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int t2o_agent_unroll_fwd(const t2o_layout* L, const float* pack_on, const float* pack_tg,
                                    const float* obs, int64_t obs_sb, int64_t obs_st, const float* h0_on,
                                    const float* h0_tg, float* q_on, float* h_on, float* q_tg, float* h_tg,
                                    int B, int T, int A, void* stream) {
  if (!L || L->kind != 0 || !pack_on || !obs || !q_on || !h_on || B < 1 || T < 1 || A < 1 ||
      L->n_ent != A)
    return T2O_EINVAL;
  AgentFwdArgs args{};
  args.L = *L;
  args.net[0] = AgentNet{pack_on, h0_on, q_on, h_on};
  int nnet = 1;
  if (pack_tg) {
    if (!q_tg || !h_tg) return T2O_EINVAL;
    args.net[1] = AgentNet{pack_tg, h0_tg, q_tg, h_tg};
    nnet = 2;
  }
  args.obs = obs;
  args.obs_sb = obs_sb;
  args.obs_st = obs_st;
  args.B = B;
  args.T = T;
  args.A = A;
  args.F = L->F;
  int rc = T2O_EUNSUPPORTED;
  T2O_DISPATCH(L->E, L->H, L->D, L->n_ent, L->FF, rc = (launch_fwd<E_, H_, D_, NE_, FF_>(args, nnet, (hipStream_t)stream)));
  return rc;
}
