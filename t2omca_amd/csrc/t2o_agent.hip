// t2o_agent.hip — TransformerAgent unrolled over a replay batch on MI355X.
//
// Reference: transf_agent.py:54-76 (+ transformer.py:40-178), called once per
// timestep by the MAC for t = 0..T of every sampled episode.  Here ONE launch
// runs the whole unroll: the agent is recurrent only through h, and every
// (episode, agent) sequence is independent, so a wave owns 16 sequences and
// carries their hidden state in registers across all timesteps (no inter-
// workgroup synchronisation at all).  A second network (the target agent) can
// run in the same launch on the same observations (blockIdx.y).
#include <cstdlib>
#include <type_traits>

#include "t2o_agent_block.hpp"
#include "t2o_agent_block_ch.hpp"
#include "t2o_dispatch.hpp"
#include "t2o_generic.hpp"
#include "t2o_layout.hpp"

using namespace t2o;

namespace {

struct AgentNet {
  const float* pack;
  const float* h0;
  float* q;
  float* h;
  float* hmid;  // [B][T][D-1][A][E] inputs of blocks 1..D-1 (may be null)
};

struct AgentFwdArgs {
  t2o_layout L;
  AgentNet net[2];
  const float* obs;
  int64_t obs_sb, obs_st;
  int B, T, A, F;
  int t0, t1;  // steps [t0, t1) of the T (outputs indexed by the full T; t0 > 0 starts from h[t0 - 1])
  int wlds;  // weights staged in LDS (set by the launcher)
  int rpw;   // rows per wave: 16, or 8 when 16-row tiles would leave SIMDs idle
};

// Rows per wave: one 16-row MFMA tile.  (8-row tiles — half the MFMA columns
// idle, twice the recurrences in flight — measured slower on config 3: the
// per-step LDS weight reads are per wave, so they double per row.)
inline int rows_per_wave(int R) { return (void)R, 16; }

constexpr int AG_FWD_WAVES = 4;  // waves per workgroup sharing one LDS copy of the weights
constexpr int AG_FWD_LOOP_T = 4;  // unrolls this short loop resident workgroups over the tiles

// Up to 8 entities the forward fits 256 VGPRs: capping it there (2 waves per
// SIMD's worth of registers) keeps the MFMA results in VGPRs instead of
// accumulation registers the compiler would otherwise copy them out of.
template <int NE>
constexpr int agent_fwd_waves_per_eu() { return NE <= 8 ? 2 : 1; }
// Observations of the next step are prefetched into registers (NE f4 per lane)
// while the current one computes.  LEAN (9-16 entities, a grid of more waves than
// SIMDs): not — the 64 prefetch registers were what kept the 16-entity forward
// above 256, and without them it runs two waves per SIMD (222 VGPRs) where the
// other wave covers the loads: 16 AGVs x 1024 episodes x T=150, agent_fwd 2.56 ->
// 2.10 ms (profiles/r5_ag16/).  A small grid keeps the prefetch (one wave per SIMD
// either way, the load latency would be exposed).
template <int NE, bool LEAN>
constexpr int agent_fwd_wpe() { return agent_fwd_waves_per_eu<NE>() > 1 || LEAN ? 2 : 1; }

// RT: runtime-entity instance (t2o_dispatch.hpp) — NE is a capacity, the real
// entity count is args.A (n_entities = n_agents on the tuned path)
template <int E, int H, int D, int NE, int FF, bool RT, bool WLDS, bool LOOP, typename WT, bool LEAN = false>
__global__ __launch_bounds__(64 * AG_FWD_WAVES) __attribute__((amdgpu_waves_per_eu(agent_fwd_wpe<NE, LEAN>())))
void agent_fwd_kernel(AgentFwdArgs args) {
  constexpr int ET = E / 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const AgentNet net = args.net[blockIdx.y];
  const t2o_layout& L = args.L;
  // the forward section of the pack lives in LDS for the whole unroll (when it fits)
  Wts<WT> P0;
  if constexpr (WLDS) {
    P0 = stage_weights(smem, net.pack, L, L.fwd_total, WT{});
    __syncthreads();
  } else {
    P0 = global_weights(net.pack, L, WT{});
  }
  P0.vol = NE <= 8;  // (Wts::vol: the 16+-entity instances run one wave per SIMD)
  const int A = args.A, F = args.F;
  const int ne = RT ? A : NE;
  const int R = args.B * A;
  // 16-row tiles, one per wave.  LOOP (a short unroll: the rollout's one step):
  // launch_fwd starts only as many workgroups as are resident and each wave loops
  // over tiles, so the weights are staged once per workgroup rather than once per
  // four tiles (rollout agent step 0.210 -> 0.179 ms fp32, 0.125 -> 0.105 ms bf16,
  // profiles/r4_agloop/); a long unroll keeps one tile per wave (the loop raised
  // the 8-entity kernel's registers 202 -> 256 with spills).  Wave-uniform: no
  // barriers after this point.
  const int tiles = (R + args.rpw - 1) / args.rpw;
  auto run_tile = [&](const int rt) {
    const int c = lane_c(), g = lane_g();
    const int row_raw = rt * args.rpw + c;
    const bool valid = c < args.rpw && row_raw < R;
    const int row = valid ? row_raw : R - 1;
    const int b = row / A, a = row % A;

    f4 h[ET];
    // a range's first step continues from the hidden state the previous range wrote
    const float* hs = args.t0 > 0 ? net.h + (((size_t)b * args.T + args.t0 - 1) * A + a) * E
                                  : net.h0 ? net.h0 + (size_t)row * E : nullptr;
#pragma unroll
    for (int t = 0; t < ET; ++t) h[t] = hs ? ld4(hs + 16 * t + 4 * g) : zero4();

    // few entities: the observations live in registers, the next step's loaded
    // while the current one computes; many entities: streamed per block in
    // chunks (t2o_agent_block_ch.hpp)
    constexpr bool CHUNK = NE > AG_CHUNK_MIN;
    constexpr int NO = CHUNK ? 1 : NE;
    constexpr bool PF = !LEAN;
    auto row_obs = [&](int step) {
      return args.obs + b * args.obs_sb + step * args.obs_st + (int64_t)a * ne * F;
    };
    auto load_obs = [&](int step, f4 (&o)[NO]) {
      const float* ob = row_obs(step);
#pragma unroll
      for (int j = 0; j < NO; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 4 * g + r;
          o[j][r] = (f < F && j < ne) ? ob[j * F + f] : 0.f;
        }
    };
    f4 on[PF ? NO : 1];
    if constexpr (!CHUNK && PF) load_obs(args.t0, on);
    for (int step = args.t0; step < args.t1; ++step) {
      const Wts<WT> P = step_view(P0);
      f4 o[NO];
      if constexpr (!CHUNK && PF) {
#pragma unroll
        for (int j = 0; j < NE; ++j) o[j] = on[j];
        if (step + 1 < args.t1) load_obs(step + 1, on);
      } else if constexpr (!CHUNK) {
        load_obs(step, o);
      }
      const ObsRow orow{row_obs(step), F, ne, RT && ne % AG_CHUNK != 0};
      f4 x[ET];
#pragma unroll
      for (int t = 0; t < ET; ++t) x[t] = h[t];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (d > 0 && net.hmid && valid) {
          float* hm = net.hmid + ((((size_t)b * args.T + step) * (D - 1) + d - 1) * A + a) * E;
#pragma unroll
          for (int t = 0; t < ET; ++t) st4(hm + 16 * t + 4 * g, x[t]);
        }
        if constexpr (CHUNK) {
          agent_block_fwd_ch<E, H, NE, FF, false>(P, L, d, h, orow, x, nullptr);
        } else {
          (void)orow;
          agent_block_fwd<E, H, NE, FF, false>(P, L, d, h, o, ne, x, nullptr);
        }
      }
      f4 q = zero4();
#pragma unroll
      for (int i = 0; i < ET; ++i) q = mma_tile(P.w + L.Wo, E, 0, i, x[i], q, P.vol);
      q += vec_t(P.v + L.bo, 0);
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
  };
  const int rt0 = blockIdx.x * AG_FWD_WAVES + wave_id();
  if constexpr (LOOP) {
    for (int rt = rt0; rt < tiles; rt += gridDim.x * AG_FWD_WAVES) run_tile(rt);
  } else {
    if (rt0 < tiles) run_tile(rt0);
  }
}

template <int E, int H, int D, int NE, int FF, bool RT, typename WT>
int launch_fwd(const AgentFwdArgs& args, int nnet, hipStream_t stream) {
  if (!kernel_layout_matches<E, H, D, FF, WT>(args.L)) return T2O_EINVAL;  // (kernels use the compile-time offsets)
  const int R = args.B * args.A;
  AgentFwdArgs a = args;
  a.rpw = rows_per_wave(R);
  const int tiles = (R + a.rpw - 1) / a.rpw;
  dim3 grid((tiles + AG_FWD_WAVES - 1) / AG_FWD_WAVES, nnet);
  size_t lds = sizeof(float) * (size_t)lds_weight_floats<WT>(args.L, args.L.fwd_total);
  a.wlds = lds <= 160 * 1024;
  if (!a.wlds) lds = 0;
  const bool loop = args.t1 - args.t0 <= AG_FWD_LOOP_T && a.wlds;
  auto kern = loop ? agent_fwd_kernel<E, H, D, NE, FF, RT, true, true, WT>
              : a.wlds ? agent_fwd_kernel<E, H, D, NE, FF, RT, true, false, WT>
                       : agent_fwd_kernel<E, H, D, NE, FF, RT, false, false, WT>;
  if constexpr (NE > 8 && NE <= AG_CHUNK_MIN) {  // (LEAN: more waves than SIMDs)
    if (!loop && a.wlds && (int64_t)tiles * nnet > 1024) kern = agent_fwd_kernel<E, H, D, NE, FF, RT, true, false, WT, true>;
  }
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (loop) {  // resident workgroups only, looping over the tiles
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 64 * AG_FWD_WAVES, lds) == hipSuccess &&
        hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && per_cu > 0 && cus > 0) {
      const unsigned cap = (unsigned)((per_cu * cus + nnet - 1) / nnet);
      if (grid.x > cap) grid.x = cap;
    }
  }
  hipLaunchKernelGGL(kern, grid, dim3(64 * AG_FWD_WAVES), lds, stream, a);
  return (int)hipGetLastError();
}


// ---------------------------------------------------------------------------
// BPTT.  One wave walks 16 sequences backwards over t; a workgroup holds
// AG_BWD_WAVES waves and one LDS copy of the forward weights (the forward
// section of the pack; transposed products read it with matvec_t).  Per step
// it recomputes the step's forward from the stored h_{t-1} and block inputs
// (hmid), then back-propagates the incoming grads (dL/dq_t, dL/dh_t from the
// mixer and from step t+1) and produces dL/dh_{t-1}.  Weight grads:
//   M, N, W1, W2   operand pairs -> tape tile (step, 16-row tile) per block;
//                  t2o_dwgemm.hpp contracts them into slab k afterwards
//   We, Wo         MFMA register blocks for the whole unroll, flushed once
//   vectors        DPP row sums + float atomics into the workgroup's slab
struct AgentBwdArgs {
  t2o_layout L, G;
  const float* pack;
  const float* obs;
  int64_t obs_sb, obs_st;
  const float* h0;
  const float* h_seq;
  const float* hmid;  // forward hmid [B][h_ts][D-1][A][E] (may be null)
  int h_ts;
  const float* gq;
  const float* gchosen;
  const int64_t* actions;
  int64_t act_sb, act_st;
  const float* gh;
  float* slabs;
  void* tape;  // [D][T * ceil(B*A/16)][TapeRec::SIZE][16] in the MFMA operand type
  float* gh0;
  int B, T, A, F;
  int rpw;  // rows per wave (rows_per_wave)
  // steps t_hi-1 .. t_lo (pipelined kernel): a range below T starts from the grad
  // wrt h[t_hi - 1] a previous range left in gcarry [B*A][E]; one above 0 leaves
  // the grad wrt h[t_lo - 1] there (gh0 gets it at t_lo = 0); only the range
  // that starts at T - 1 clears the slab regions the flushes add into
  int t_lo, t_hi;
  float* gcarry;
};

constexpr int AG_BWD_WAVES = 2;  // (each wave needs a SIMD's full 512-register file)

template <int E, int H, int D, int NE, int FF, bool RT, typename WT>
__global__ __launch_bounds__(64 * AG_BWD_WAVES) void agent_bwd_kernel(AgentBwdArgs args) {
  constexpr int ET = E / 16;
  constexpr int STAGE = StageDims<1>::FLOATS;
  using Rec = TapeRec<E, H, FF>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const t2o_layout& L = args.L;
  const t2o_layout& G = args.G;
  // the forward section of the pack; transposed products read it transposed (matvec_tr)
  const int64_t nw = L.fwd_total;
  const int lds_w = (int)((lds_weight_floats<WT>(L, nw) + 15) / 16 * 16);
  float* stage = smem + lds_w + wave_id() * STAGE;
  float* gs = args.slabs + (size_t)blockIdx.x * G.grad_total;
  Wts<WT> P0 = stage_weights(smem, args.pack, L, nw, WT{});
  P0.vol = NE <= 8;  // (Wts::vol)
  zero_flushed_regions(gs, G, false);  // (full record: the contraction writes M / N)
  __syncthreads();

  const int A = args.A, F = args.F, T = args.T;
  const int ne = RT ? A : NE;
  const int R = args.B * A;
  const int rt = blockIdx.x * AG_BWD_WAVES + wave_id();
  const int c = lane_c(), g = lane_g();
  const int row_raw = rt * args.rpw + c;
  const bool valid = c < args.rpw && row_raw < R;
  const int row = valid ? row_raw : R - 1;
  const int b = row / A, a = row % A;
  const size_t tiles_per_step = (size_t)(R + 15) / 16;
  const size_t ntiles = (size_t)T * tiles_per_step;

  f4 gWe[ET][1], gWo[1][ET];
#pragma unroll
  for (int t = 0; t < ET; ++t) gWe[t][0] = gWo[0][t] = zero4();
  // per-lane partial sums over the wave's steps, reduced once at the end:
  // LN2 vectors of every block, embedding bias, head bias
  f4 ln2[D][2 * ET], gbe[ET], gbo = zero4();
#pragma unroll
  for (int t = 0; t < ET; ++t) {
    gbe[t] = zero4();
#pragma unroll
    for (int d = 0; d < D; ++d) ln2[d][t] = ln2[d][ET + t] = zero4();
  }
  if (rt * args.rpw < R) {
    f4 gh_rec[ET];
#pragma unroll
    for (int t = 0; t < ET; ++t) gh_rec[t] = zero4();
    for (int step = T - 1; step >= 0; --step) {
      const Wts<WT> P = step_view(P0);
      f4 h[ET];
      const float* hp = step == 0 ? args.h0 : args.h_seq + (((size_t)b * args.h_ts + step - 1) * A + a) * E;
      if (step == 0 && args.h0) hp = args.h0 + (size_t)row * E;
#pragma unroll
      for (int t = 0; t < ET; ++t) h[t] = hp ? ld4(hp + 16 * t + 4 * g) : zero4();
      const float* ob = args.obs + b * args.obs_sb + step * args.obs_st + (int64_t)a * ne * F;
      constexpr bool CHUNK = NE > AG_CHUNK_MIN;  // many entities: streamed per block (t2o_agent_block_ch.hpp)
      constexpr int NO = CHUNK ? 1 : NE;
      const ObsRow orow{ob, F, ne, RT && ne % AG_CHUNK != 0};
      f4 o[NO];
      if constexpr (!CHUNK) {
#pragma unroll
        for (int j = 0; j < NE; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int f = 4 * g + r;
            o[j][r] = (f < F && j < ne) ? ob[j * F + f] : 0.f;
          }
      }
      // external grads of this step
      const size_t sidx = ((size_t)b * T + step) * A + a;
      f4 gq = zero4();
      if (args.gq) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * g + r < L.NA) gq[r] = args.gq[sidx * L.NA + 4 * g + r];
      }
      if (args.gchosen) {
        const int64_t act = args.actions[b * args.act_sb + step * args.act_st + a];
        const float gc = args.gchosen[sidx];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * g + r == act) gq[r] += gc;
      }
      f4 gx[ET];
#pragma unroll
      for (int t = 0; t < ET; ++t) {
        gx[t] = gh_rec[t];
        if (args.gh) gx[t] += ld4(args.gh + sidx * E + 16 * t + 4 * g);
      }
      if (!valid) {
        gq = zero4();
#pragma unroll
        for (int t = 0; t < ET; ++t) gx[t] = zero4();
      }
      // inputs of every block: stored by the forward, else recomputed
      f4 xs[D][ET];
#pragma unroll
      for (int t = 0; t < ET; ++t) xs[0][t] = h[t];
      if (args.hmid) {
#pragma unroll
        for (int d = 1; d < D; ++d) {
          const float* hm = args.hmid + ((((size_t)b * args.h_ts + step) * (D - 1) + d - 1) * A + a) * E;
#pragma unroll
          for (int t = 0; t < ET; ++t) xs[d][t] = ld4(hm + 16 * t + 4 * g);
        }
      } else {
#pragma unroll
        for (int d = 0; d + 1 < D; ++d) {
          f4 x[ET];
#pragma unroll
          for (int t = 0; t < ET; ++t) x[t] = xs[d][t];
          if constexpr (CHUNK) agent_block_fwd_ch<E, H, NE, FF, false>(P, L, d, h, orow, x, nullptr);
          else agent_block_fwd<E, H, NE, FF, false>(P, L, d, h, o, ne, x, nullptr);
#pragma unroll
          for (int t = 0; t < ET; ++t) xs[d + 1][t] = x[t];
        }
      }
      f4 gh_in[ET];
#pragma unroll
      for (int t = 0; t < ET; ++t) gh_in[t] = zero4();
#pragma unroll
      for (int d = D - 1; d >= 0; --d) {
        typename std::conditional<CHUNK, AgentCacheCh<E, H, NE, FF>, AgentCache<E, H, NE, FF>>::type cache;
        f4 x[ET];
#pragma unroll
        for (int t = 0; t < ET; ++t) x[t] = xs[d][t];
        if constexpr (CHUNK) agent_block_fwd_ch<E, H, NE, FF, true>(P, L, d, h, orow, x, &cache);
        else agent_block_fwd<E, H, NE, FF, true>(P, L, d, h, o, ne, x, &cache);
        if (d == D - 1) {  // q = Wo x + bo
          dw_accumulate_regs<1, ET, sizeof(WT) == 2>(gWo, &gq, x, stage);
          gbo += gq;
          f4 t1[ET];
          matvec_tr<ET, 1>(P, L.Wo, E, L.WoT, 16, &gq, t1);
#pragma unroll
          for (int t = 0; t < ET; ++t) gx[t] += t1[t];
        }
        // padding rows write their (zero-gradient) records too: a tile is written whole
        WT* rec = static_cast<WT*>(args.tape) + ((size_t)d * ntiles + (size_t)step * tiles_per_step + rt) * Rec::SIZE * 16;
        if constexpr (CHUNK)
          agent_block_bwd_ch<E, H, NE, FF>(P, L, G, gs, rec, stage, d, h, orow, cache, gx, gh_in, gbe, gWe, ln2[d]);
        else
          agent_block_bwd<E, H, NE, FF>(P, L, G, gs, rec, stage, d, h, o, cache, gx, gh_in, gbe, gWe, ln2[d]);
      }
#pragma unroll
      for (int t = 0; t < ET; ++t) gh_rec[t] = gx[t] + gh_in[t];
    }
    if (args.gh0 && valid) {
#pragma unroll
      for (int t = 0; t < ET; ++t) st4(args.gh0 + (size_t)row * E + 16 * t + 4 * g, gh_rec[t]);
    }
  }
  flush_in_wave_order([&] {
    if (rt * args.rpw < R) {
      flush_tiles_g<ET, 1>(gs + G.We, 16, gWe);
      flush_tiles_g<1, ET>(gs + G.Wo, E, gWo);
      vec_accumulate_g<ET>(gs + G.be, gbe);
      vec_accumulate_g<1>(gs + G.bo, &gbo);
      ln2_flush<E, D>(gs, G, ln2);
    }
  });
}

// ---------------------------------------------------------------------------
// BPTT with the blocks on separate waves (depth 2, block inputs stored by the
// forward).  The single-wave kernel above issues, per step, the forward
// recompute and the backward of both blocks back to back on one SIMD, and with
// one 16-row tile per wave (8,192 rows = 512 waves) it leaves half the SIMDs
// idle.  Here each tile gets two waves: wave "d" owns block d (its forward
// recompute, cache and backward) and the two interleave so that one's recompute
// overlaps the other's backward (phases separated by the pair's barrier,
// t2o_common.hpp PairBarrier):
//   block-1 wave:  fwd(T-1) | bwd(T-1) | fwd(T-2) | bwd(T-2) | ...
//   block-0 wave:     -     | fwd(T-1) | bwd(T-1) | fwd(T-2) | ...
// Per step the dependent work is bwd1 -> bwd0 -> bwd1 ..., exchanged through
// LDS (per lane: grad wrt the block-1 input and the block-1 key/value grad of h,
// 1 -> 0; the recurrent grad wrt h_{t-1}, 0 -> 1), one pair barrier per
// phase.  The backward of a block is the same code as in the single-wave
// kernel, so records, slabs and the head grads are identical in meaning.
// T2O_AGENT_BWD=single selects the single-wave kernel (A/B timing, parity cross-check)
inline bool agent_bwd_single_wave() {  // (read per call: a test switches it within one process)
  const char* e = getenv("T2O_AGENT_BWD");
  return e && e[0] == 's';
}

constexpr int AGP_TILES = AG_BWD_WAVES;  // tiles per workgroup (same slab count as the single-wave kernel)

template <int E>
constexpr int agp_xch_floats() { return 3 * (E / 16) * 64 * 4; }

// the pipelined kernel keeps dM / dN in registers (tape record TapeRecA) in bf16
// up to 8 entities (beyond, 96 more accumulator registers spill); otherwise it
// tapes the full record
template <int E, int H, int NE, typename WT>
constexpr bool agp_acc() { return sizeof(WT) == 2 && NE <= 8; }
template <int E, int H, int NE, typename WT>
constexpr int agp_stage_floats() {
  return agp_acc<E, H, NE, WT>() ? AgentAccTiles<E, H>::N * 128 : StageDims<1>::FLOATS;
}

template <int E, int H, int D, int NE, int FF, bool RT, typename WT>
// (The body lives in the kernel itself.  Round 3 moved it into a device function
// taking the args and layouts by reference, to be callable with a compile-time
// layout: the compiler then spilled 28 B per lane to scratch, one reload in the
// step loop, and agent_bwd went 0.543 -> 0.604 ms — bisected, profiles/r4_bisect/.
// Compile-time offsets had measured slower here anyway: 0.623 -> 0.643 ms,
// profiles/r3_ab6/.)
__global__ __launch_bounds__(64 * 2 * AGP_TILES) void agent_bwd_pipe_kernel(AgentBwdArgs args) {
  const t2o_layout& L = args.L;
  const t2o_layout& G = args.G;
  static_assert(D == 2, "one wave per block of a depth-2 stack");
  constexpr int ET = E / 16, HET = H * ET;
  constexpr bool BF = sizeof(WT) == 2;
  constexpr bool CHUNK = NE > AG_CHUNK_MIN;
  constexpr int NO = CHUNK ? 1 : NE;
  // bf16, entities in registers: dM / dN accumulate in registers (lean record)
  constexpr bool ACC = agp_acc<E, H, NE, WT>();
  constexpr int STAGE = agp_stage_floats<E, H, NE, WT>();
  using Rec = typename std::conditional<ACC, TapeRecA<E, H, FF>, TapeRec<E, H, FF>>::type;
  // lean cache (half the registers of the one-wave kernel's; X, Z, Y records
  // written by the recompute phase) unless the entities are streamed in chunks
  using Cache = typename std::conditional<CHUNK, AgentCacheCh<E, H, NE, FF>, AgentCacheLean<E, H, NE, FF>>::type;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const int64_t nw = L.fwd_total;
  const int lds_w = (int)((lds_weight_floats<WT>(L, nw) + 15) / 16 * 16);
  // wave-uniform by construction; readfirstlane tells the compiler, so the block's
  // layout offsets (L.M[d] ...) are scalar loads, not per-lane global loads
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  // the block this wave owns.  Waves w and w + 4 share a SIMD: with four pairs,
  // pairs 2-3 swap their block roles so every SIMD holds one block-0 and one
  // block-1 wave (the two phases of a barrier interval differ in cost)
#ifndef T2O_PIPE_NO_SIMD_MIX
  const int d = (w ^ (w >> 2)) & 1;
#else
  const int d = w & 1;
#endif
  const int tl = w >> 1; // tile within the workgroup
  const t2o_layout Lb = block_view(L, d), Gb = block_view(G, d);
  float* stage = smem + lds_w + w * STAGE;
  f4* xch = reinterpret_cast<f4*>(smem + lds_w + 2 * AGP_TILES * STAGE + tl * agp_xch_floats<E>());
  const int lane = threadIdx.x & 63;
  float* gs = args.slabs + (size_t)blockIdx.x * G.grad_total;
  Wts<WT> P0 = stage_weights(smem, args.pack, L, nw, WT{});
  P0.vol = NE <= 8;  // (Wts::vol: 16+ entities measured slower with volatile reads)
  if (args.t_hi == args.T) zero_flushed_regions(gs, G, ACC);  // (lean record: dM / dN flushed from registers)
  int* const flags = reinterpret_cast<int*>(smem + lds_w + 2 * AGP_TILES * STAGE + AGP_TILES * agp_xch_floats<E>());
  if (threadIdx.x < PAIR_FLAG_FLOATS) flags[threadIdx.x] = 0;
  __syncthreads();
  // the tile's two waves synchronise pairwise (t2o_common.hpp PairBarrier)
  PairBarrier pb = PairBarrier::make(flags, w);

  const int A = args.A, F = args.F, T = args.T;
  const int ne = RT ? A : NE;
  const bool tail = RT && ne % AG_CHUNK != 0;
  const int R = args.B * A;
  const int rt = blockIdx.x * AGP_TILES + tl;
  const int c = lane_c(), g = lane_g();
  const bool tile_ok = rt * 16 < R;
  const int row_raw = rt * 16 + c;
  const bool valid = row_raw < R;
  const int row = valid ? row_raw : R - 1;
  const int b = row / A, a = row % A;
  const size_t tiles_per_step = (size_t)(R + 15) / 16;
  const size_t ntiles = (size_t)T * tiles_per_step;
  // exchange slots: 0 grad wrt block-1 input, 1 block-1 K/V grad of h, 2 grad wrt h_{t-1}
  auto xput = [&](int k, const f4* v) {
#pragma unroll
    for (int t = 0; t < ET; ++t) xch[(k * ET + t) * 64 + lane] = v[t];
  };
  auto xget = [&](int k, f4* v) {
#pragma unroll
    for (int t = 0; t < ET; ++t) v[t] = xch[(k * ET + t) * 64 + lane];
  };

  f4 gWe[ET][1], gWo[1][ET], gbe[ET], ln2[2 * ET], gbo = zero4();
#pragma unroll
  for (int t = 0; t < ET; ++t) {
    gWe[t][0] = gWo[0][t] = gbe[t] = zero4();
    ln2[t] = ln2[ET + t] = zero4();
  }
  f4 gM[HET][ET], gN[ET][HET];  // ACC: this wave's block's dM, dN over its tile and the unroll
#pragma unroll
  for (int i = 0; i < HET; ++i)
#pragma unroll
    for (int t = 0; t < ET; ++t) gM[i][t] = gN[t][i] = zero4();
  if constexpr (ACC) {  // the first recompute's deferred contractions then add zeros
    for (int i = lane; i < STAGE; i += 64) stage[i] = 0.f;
  }
  // Both roles run the same loop body "recompute step; barrier; backward step;
  // barrier"; the block-0 wave starts one barrier late, so its recompute of a
  // step overlaps the block-1 backward of the same step and its backward the
  // block-1 recompute of the next (earlier) one.  The cache lives within one
  // iteration.
  auto load_fwd_inputs = [&](int step, f4* hh, f4 (&oo)[NO], f4* xx) {
    const float* hp = step == 0 ? (args.h0 ? args.h0 + (size_t)row * E : nullptr)
                                : args.h_seq + (((size_t)b * args.h_ts + step - 1) * A + a) * E;
#pragma unroll
    for (int t = 0; t < ET; ++t) hh[t] = hp ? ld4(hp + 16 * t + 4 * g) : zero4();
    if constexpr (!CHUNK) {
      const float* obp = args.obs + b * args.obs_sb + step * args.obs_st + (int64_t)a * ne * F;
#pragma unroll
      for (int j = 0; j < NE; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 4 * g + r;
          oo[j][r] = (f < F && j < ne) ? obp[j * F + f] : 0.f;
        }
    }
    if (d == 1) {  // (block 0's input is h itself: copied where used, never here —
                   // touching a register with a load in flight waits for it)
      const float* hm = args.hmid + (((size_t)b * args.h_ts + step) * (D - 1) * A + a) * E;
#pragma unroll
      for (int t = 0; t < ET; ++t) xx[t] = ld4(hm + 16 * t + 4 * g);
    }
  };
  // A step's inputs are loaded at the end of the previous (later) step's
  // backward phase, after its last use of them: the loads are then in flight
  // through the barrier wait instead of stalling the start of the recompute.
  // The block-1 wave's output grads (dL/dh_t from the mixer, dL/dq_t; the
  // recurrent part of dL/dh_t comes from block 0) are loaded raw with them and
  // combined where the backward uses them.
  f4 h[ET], o[NO], xo[ET], ghx[ET], gqv = zero4();
  float gc = 0.f;
  int64_t act = -1;
  auto load_step = [&](int step) {
    load_fwd_inputs(step, h, o, xo);
    if (d == 1) {
      const size_t sidx = ((size_t)b * T + step) * A + a;
#pragma unroll
      for (int t = 0; t < ET; ++t) ghx[t] = args.gh ? ld4(args.gh + sidx * E + 16 * t + 4 * g) : zero4();
      if (args.gq) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * g + r < L.NA) gqv[r] = args.gq[sidx * L.NA + 4 * g + r];
      }
      if (args.gchosen) {
        act = args.actions[b * args.act_sb + step * args.act_st + a];
        gc = args.gchosen[sidx];
      }
    }
  };
  const int t_lo = args.t_lo, t_hi = args.t_hi;
  load_step(t_hi - 1);
  if (d == 0) pb.sync();
  for (int step = t_hi - 1; step >= t_lo; --step) {
#ifdef T2O_TIMELINE
    T2O_STAMP(2 * (T - 1 - step), 0);
#endif
    Cache cache;
    const float* ob = args.obs + b * args.obs_sb + step * args.obs_st + (int64_t)a * ne * F;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      T2O_MARK(0);
#ifdef T2O_TIMELINE
      if (ph == 0) T2O_STAMP(2 * (T - 1 - step), 1);
#endif
      const Wts<WT> P = step_view(P0);
      WT* const tile = static_cast<WT*>(args.tape) +
                       ((size_t)d * ntiles + (size_t)step * tiles_per_step + rt) * Rec::SIZE * 16;
      if (ph == 0) {
#if defined(T2O_PHASE_PROF) && !defined(T2O_TIMELINE)  // (timelines: no forced drain)
        __builtin_amdgcn_s_waitcnt(0);
#endif
        T2O_MARK(1);
        if (d == 0) {
#pragma unroll
          for (int t = 0; t < ET; ++t) xo[t] = h[t];
        }
        if constexpr (CHUNK) agent_block_fwd_ch<E, H, NE, FF, true>(P, Lb, 0, h, ObsRow{ob, F, ne, tail}, xo, &cache);
        else if constexpr (ACC)
          agent_block_fwd_acc<E, H, NE, FF>(P, Lb, 0, h, o, ne, xo, cache,
                                            MaskedRec<WT>(tile, tile_ok ? 16 : 0, Rec::SIZE), stage, gM, gN, gWe);
        else agent_block_fwd_lean<E, H, NE, FF>(P, Lb, 0, h, o, ne, xo, cache,
                                                MaskedRec<WT>(tile, tile_ok ? 16 : 0, Rec::SIZE));
      } else {
        f4 gx[ET], ghi[ET];
        if (d == 1) {
          f4 gq = gqv;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (4 * g + r == act) gq[r] += gc;
          if (step < t_hi - 1) xget(2, gx);
          else if (t_hi < T) {  // the grad wrt h[t_hi - 1] from the range after this one
#pragma unroll
            for (int t = 0; t < ET; ++t) gx[t] = ld4(args.gcarry + (size_t)row * E + 16 * t + 4 * g);
          } else {
#pragma unroll
            for (int t = 0; t < ET; ++t) gx[t] = zero4();
          }
#pragma unroll
          for (int t = 0; t < ET; ++t) gx[t] += ghx[t];
          if (!valid) {
            gq = zero4();
#pragma unroll
            for (int t = 0; t < ET; ++t) gx[t] = zero4();
          }
          // q = Wo x + bo on the stack output
          dw_accumulate_regs<1, ET, BF>(gWo, &gq, xo, stage);
          gbo += gq;
          f4 t1[ET];
          matvec_tr<ET, 1>(P, L.Wo, E, L.WoT, 16, &gq, t1);
#pragma unroll
          for (int t = 0; t < ET; ++t) {
            gx[t] += t1[t];
            ghi[t] = zero4();
          }
        } else {
          xget(0, gx);
          xget(1, ghi);
        }
#if defined(T2O_PHASE_PROF) && !defined(T2O_TIMELINE)  // (timelines: no forced drain)
        __builtin_amdgcn_s_waitcnt(0);
#endif
        T2O_MARK(1);
        if constexpr (CHUNK)
          agent_block_bwd_ch<E, H, NE, FF>(P, Lb, Gb, gs, tile_ok ? tile : nullptr, stage, 0, h, ObsRow{ob, F, ne, tail}, cache,
                                           gx, ghi, gbe, gWe, ln2);
        else if constexpr (ACC)
          agent_block_bwd_acc<E, H, NE, FF>(P, Lb, gs, MaskedRec<WT>(tile, tile_ok ? 16 : 0, Rec::SIZE), stage, 0, h,
                                            o, cache, gx, ghi, gbe, gWe, ln2, gM, gN);
        else
          agent_block_bwd_lean<E, H, NE, FF>(P, Lb, gs, MaskedRec<WT>(tile, tile_ok ? 16 : 0, Rec::SIZE), stage, 0, h,
                                             o, cache, gx, ghi, gbe, gWe, ln2);
        if (d == 1) {
          xput(0, gx);
          xput(1, ghi);
        } else {
          f4 grec[ET];
#pragma unroll
          for (int t = 0; t < ET; ++t) grec[t] = gx[t] + ghi[t];
          xput(2, grec);
          float* const gout = step > 0 ? args.gcarry : args.gh0;
          if (step == t_lo && gout && valid) {
#pragma unroll
            for (int t = 0; t < ET; ++t) st4(gout + (size_t)row * E + 16 * t + 4 * g, grec[t]);
          }
        }
        if (step > t_lo) load_step(step - 1);
      }
      T2O_MARK(3);
#ifdef T2O_TIMELINE
      T2O_STAMP(2 * (T - 1 - step) + ph, 2 * (1 - ph));
#endif
      pb.sync();
      T2O_MARK(4);
#ifdef T2O_TIMELINE
      T2O_STAMP(2 * (T - 1 - step) + ph, 3 - 2 * ph);
#else
      T2O_PROF_SAVE((T - 1 - step) * 2 + ph, 4);
#endif
    }
  }
  if (d == 1) pb.sync();
  if constexpr (ACC) agent_dw_deferred<E, H>(stage, gM, gN, gWe);  // the last backward phase's
  flush_in_wave_order([&] {
    if (tile_ok) {
      if constexpr (ACC) {
        flush_tiles_g<HET, ET>(gs + Gb.M[0], E, gM);
        flush_tiles_g<ET, HET>(gs + Gb.N[0], H * E, gN);
      }
      flush_tiles_g<ET, 1>(gs + G.We, 16, gWe);
      vec_accumulate_g<ET>(gs + G.be, gbe);
      vec_accumulate_g<ET>(gs + Gb.g2[0], &ln2[0]);
      vec_accumulate_g<ET>(gs + Gb.n2[0], &ln2[ET]);
      if (d == 1) {
        flush_tiles_g<1, ET>(gs + G.Wo, E, gWo);
        vec_accumulate_g<1>(gs + G.bo, &gbo);
      }
    }
  });
}

template <int E, int H, int D, int NE, int FF, typename WT>
size_t bwd_pipe_lds_bytes(const t2o_layout& L) {
  const int64_t nw = L.fwd_total;
  return sizeof(float) * ((size_t)(lds_weight_floats<WT>(L, nw) + 15) / 16 * 16 +
                          2 * AGP_TILES * agp_stage_floats<E, H, NE, WT>() + AGP_TILES * agp_xch_floats<E>() +
                          PAIR_FLAG_FLOATS);
}

// which BPTT kernel launch_bwd picks: the pipelined one (depth 2, block inputs
// stored by the forward, LDS fits, no T2O_AGENT_BWD=single)
template <int E, int H, int D, int NE, int FF, bool RT, typename WT>
bool bwd_uses_pipe(const t2o_layout& L, bool has_hmid) {
  if constexpr (D == 2) return has_hmid && bwd_pipe_lds_bytes<E, H, D, NE, FF, WT>(L) <= 160 * 1024 && !agent_bwd_single_wave();
  return false;
}

template <int E, int H, int D, int NE, int FF, bool RT, typename WT>
int bwd_tape_format(const t2o_layout& L, bool has_hmid) {
  return bwd_uses_pipe<E, H, D, NE, FF, RT, WT>(L, has_hmid) && agp_acc<E, H, NE, WT>() ? 1 : 0;
}

template <int E, int H, int D, int NE, int FF, bool RT, typename WT>
int launch_bwd(AgentBwdArgs& args, int max_slabs, int* nslab, hipStream_t stream) {
  if (!kernel_layout_matches<E, H, D, FF, WT>(args.L)) return T2O_EINVAL;  // (kernels use the compile-time offsets)
  const int R = args.B * args.A;
  args.rpw = rows_per_wave(R);
  const int tiles = (R + args.rpw - 1) / args.rpw;
  const int grid = (tiles + AG_BWD_WAVES - 1) / AG_BWD_WAVES;
  if (grid > max_slabs) return T2O_EINVAL;
  if constexpr (D == 2) {
    const size_t lds = bwd_pipe_lds_bytes<E, H, D, NE, FF, WT>(args.L);
    if (bwd_uses_pipe<E, H, D, NE, FF, RT, WT>(args.L, args.hmid != nullptr)) {
      auto kern = agent_bwd_pipe_kernel<E, H, D, NE, FF, RT, WT>;
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * 2 * AGP_TILES), lds, stream, args);
      *nslab = grid;
      return (int)hipGetLastError();
    }
  }
  if (args.t_lo != 0 || args.t_hi != args.T) return T2O_EUNSUPPORTED;  // (step ranges: the pipelined kernel)
  const int64_t nw = args.L.fwd_total;
  const size_t lds =
      sizeof(float) * ((size_t)(lds_weight_floats<WT>(args.L, nw) + 15) / 16 * 16 + AG_BWD_WAVES * StageDims<1>::FLOATS);
  auto kern = agent_bwd_kernel<E, H, D, NE, FF, RT, WT>;
  if (lds > 160 * 1024) return T2O_EUNSUPPORTED;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * AG_BWD_WAVES), lds, stream, args);
  *nslab = grid;
  return (int)hipGetLastError();
}

}  // namespace

static int agent_fwd_impl(const t2o_layout* L, const float* pack_on, const float* pack_tg,
                                          const float* obs, int64_t obs_sb, int64_t obs_st, const float* h0_on,
                                          const float* h0_tg, float* q_on, float* h_on, float* hmid_on,
                                          float* q_tg, float* h_tg, float* hmid_tg, int B, int T, int A, int t0,
                                          int t1, void* stream) {
  if (!L || L->kind != 0 || !pack_on || !obs || !q_on || !h_on || B < 1 || T < 1 || A < 1 ||
      (!L->generic && L->n_ent != A) || t0 < 0 || t1 > T || t0 >= t1)
    return T2O_EINVAL;
  if (L->generic) {
    if (t0 != 0 || t1 != T) return T2O_EUNSUPPORTED;
    return gen_agent_unroll_fwd(L, pack_on, pack_tg, obs, obs_sb, obs_st, h0_on, h0_tg, q_on, h_on, hmid_on, q_tg,
                                h_tg, hmid_tg, B, T, A, (hipStream_t)stream);
  }
  AgentFwdArgs args{};
  args.L = *L;
  args.net[0] = AgentNet{pack_on, h0_on, q_on, h_on, hmid_on};
  int nnet = 1;
  if (pack_tg) {
    if (!q_tg || !h_tg) return T2O_EINVAL;
    args.net[1] = AgentNet{pack_tg, h0_tg, q_tg, h_tg, hmid_tg};
    nnet = 2;
  }
  args.obs = obs;
  args.obs_sb = obs_sb;
  args.obs_st = obs_st;
  args.B = B;
  args.T = T;
  args.A = A;
  args.F = L->F;
  args.t0 = t0;
  args.t1 = t1;
  int rc = T2O_EUNSUPPORTED;
  T2O_DISPATCH_AGENT(L->E, L->H, L->D, L->n_ent, L->FF,
                     rc = (L->prec ? launch_fwd<E_, H_, D_, NE_, FF_, RT_, __bf16>(args, nnet, (hipStream_t)stream)
                                   : launch_fwd<E_, H_, D_, NE_, FF_, RT_, float>(args, nnet, (hipStream_t)stream)));
  return rc;
}

static int agent_bwd_impl(const t2o_layout* L, const float* pack, const float* obs, int64_t obs_sb,
                                          int64_t obs_st, const float* h0, const float* h_seq, const float* hmid,
                                          int h_ts, const float* gq, const float* gchosen, const int64_t* actions,
                                          int64_t act_sb, int64_t act_st, const float* gh, float* gslabs,
                                          int max_slabs, int* nslab, void* tape, float* gh0, float* gcarry, int B,
                                          int T, int A, int t_lo, int t_hi, void* stream) {
  if (!L || L->kind != 0 || !pack || !obs || !h_seq || !gslabs || !nslab || !tape || B < 1 || T < 1 || A < 1 ||
      (!L->generic && L->n_ent != A) || h_ts < T || (gchosen && !actions) || t_lo < 0 || t_hi > T ||
      t_lo >= t_hi || ((t_lo > 0 || t_hi < T) && !gcarry))
    return T2O_EINVAL;
  if (L->generic && (t_lo != 0 || t_hi != T)) return T2O_EUNSUPPORTED;
  if (L->generic)
    return gen_agent_unroll_bwd(L, pack, obs, obs_sb, obs_st, h0, h_seq, hmid, h_ts, gq, gchosen, actions, act_sb,
                                act_st, gh, gslabs, max_slabs, nslab, tape, gh0, B, T, A, (hipStream_t)stream);
  AgentBwdArgs args{};
  args.L = *L;
  grad_layout(*L, args.G);
  args.pack = pack;
  args.obs = obs;
  args.obs_sb = obs_sb;
  args.obs_st = obs_st;
  args.h0 = h0;
  args.h_seq = h_seq;
  args.hmid = hmid;
  args.h_ts = h_ts;
  args.gq = gq;
  args.gchosen = gchosen;
  args.actions = actions;
  args.act_sb = act_sb;
  args.act_st = act_st;
  args.gh = gh;
  args.slabs = gslabs;
  args.tape = tape;
  args.gh0 = gh0;
  args.B = B;
  args.T = T;
  args.A = A;
  args.F = L->F;
  args.t_lo = t_lo;
  args.t_hi = t_hi;
  args.gcarry = gcarry;
  int rc = T2O_EUNSUPPORTED;
  T2O_DISPATCH_AGENT(L->E, L->H, L->D, L->n_ent, L->FF,
                     rc = (L->prec ? launch_bwd<E_, H_, D_, NE_, FF_, RT_, __bf16>(args, max_slabs, nslab, (hipStream_t)stream)
                                   : launch_bwd<E_, H_, D_, NE_, FF_, RT_, float>(args, max_slabs, nslab, (hipStream_t)stream)));
  return rc;
}

extern "C" int t2o_agent_unroll_fwd(const t2o_agent_fwd_args* a, void* stream) {
  if (!a) return T2O_EINVAL;
  return agent_fwd_impl(a->L, a->pack_on, a->pack_tg, a->obs, a->obs_sb, a->obs_st, a->h0_on, a->h0_tg, a->q_on,
                        a->h_on, a->hmid_on, a->q_tg, a->h_tg, a->hmid_tg, a->B, a->T, a->A, a->t0,
                        a->t1 > 0 ? a->t1 : a->T, stream);
}

extern "C" int t2o_agent_unroll_bwd(const t2o_agent_bwd_args* a, void* stream) {
  if (!a) return T2O_EINVAL;
  return agent_bwd_impl(a->L, a->pack, a->obs, a->obs_sb, a->obs_st, a->h0, a->h_seq, a->hmid, a->h_ts, a->gq,
                        a->gchosen, a->actions, a->act_sb, a->act_st, a->gh, a->gslabs, a->max_slabs, a->nslab, a->tape,
                        a->gh0, a->gcarry, a->B, a->T, a->A, a->t_lo, a->t_hi > 0 ? a->t_hi : a->T, stream);
}

// diagnostic builds only (-DT2O_PHASE_PROF, tools/phase_prof.py)
T2O_PROF_READER(t2o_prof_read_agent)

extern "C" int t2o_agent_bwd_tape_format(const t2o_layout* L, int has_hmid) {
  if (!L || L->kind != 0) return T2O_EINVAL;
  if (L->generic) return 0;
  int fmt = 0;
  T2O_DISPATCH_AGENT(L->E, L->H, L->D, L->n_ent, L->FF,
                     fmt = (L->prec ? bwd_tape_format<E_, H_, D_, NE_, FF_, RT_, __bf16>(*L, has_hmid != 0)
                                    : bwd_tape_format<E_, H_, D_, NE_, FF_, RT_, float>(*L, has_hmid != 0)));
  return fmt;
}

extern "C" int t2o_agent_bwd_ranges(const t2o_layout* L, int has_hmid) {
  if (!L || L->kind != 0) return T2O_EINVAL;
  if (L->generic) return 0;
  int ok = 0;
  T2O_DISPATCH_AGENT(L->E, L->H, L->D, L->n_ent, L->FF,
                     ok = (L->prec ? bwd_uses_pipe<E_, H_, D_, NE_, FF_, RT_, __bf16>(*L, has_hmid != 0)
                                   : bwd_uses_pipe<E_, H_, D_, NE_, FF_, RT_, float>(*L, has_hmid != 0)));
  return ok ? 1 : 0;
}

extern "C" int t2o_agent_bwd_max_slabs(int B, int A) {
  const int rpw = rows_per_wave(B * A);
  const int tiles = (B * A + rpw - 1) / rpw;
  return (tiles + AG_BWD_WAVES - 1) / AG_BWD_WAVES;
}
