// t2o_mixer.hip — TransformerMixer unrolled over a replay batch on MI355X.
//
// Reference: n_transf_mixer.py:55-91 driven by the learner once per timestep
// with the recurrent hyper-weight tokens (n_transf_mixer.py:69,91).  One wave
// owns one episode for the whole unroll (episodes are independent; the
// recurrence is only over the 3 hyper tokens), so a launch needs no
// inter-workgroup synchronisation.  The learner's Q selection is fused into
// the mixer's input read:
//   qmode 0  qvals given directly                      [b][t][a]
//   qmode 1  chosen-action Q  gather(Q[:, t], actions)  (online mixer)
//   qmode 2  double-Q         Q_tgt[argmax(Q_on masked by avail)] (target mixer)
// per-product weight swizzle (t2o_common.hpp matvec): these kernels are register-bound
#define T2O_SWZ_HOIST 0
#include "t2o_dispatch.hpp"
#include "t2o_generic.hpp"
#include "t2o_layout.hpp"
#include "t2o_mixer_block.hpp"
#include "t2o_mixer_parts.hpp"

using namespace t2o;

namespace {
// RT (t2o_dispatch.hpp RTM_): 0 exact agent count A + abs head; 1 runtime-agent
// instance (A a capacity, args.na the agent count) + runtime head; 2 exact A +
// runtime head (L.pos_func)
// LB: the launch bound.  512 (8 waves, two per SIMD: 256 registers a wave); 256 for
// the multi-tile mixers when the launch holds at most four waves per workgroup — the
// LDS then admits one workgroup per CU, i.e. one wave per SIMD, and the wave may take
// the whole register file (at 64 AGVs the 256-register build spilled 0.5-1.9 KB a lane)
template <int E, int H, int D, int A, int FF, int RT, bool WLDS, typename WT, int LB = 512>
__global__ __launch_bounds__(LB) void mixer_fwd_kernel(MixerFwdArgs args) {
  using Dm = MixDims<E, A>;
  constexpr int ET = E / 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const int w = wave_id();
  const MixerNet n = args.net[blockIdx.y];
  // bf16: the pack offsets as compile-time constants (t2o_layout.hpp kernel_layout,
  // as the pipelined BPTT reads them; the launcher checks they match)
  const t2o_layout L = kernel_layout<E, H, D, FF, WT>(args.L);
  const int na = RT == 1 ? args.na : A, nq = na + 3, lk = 2 * na + 3;
  const int pf = RT ? L.pos_func : T2O_POS_ABS;  // the mixer head's positivity function
  const float pb = RT ? L.pos_beta : 1.f;
  // forward weights in LDS for the unroll when they fit beside the per-wave buffers
  const int lds_w = WLDS ? (int)((lds_weight_floats<WT>(L, L.fwd_total) + 15) / 16 * 16) : 0;
  Wts<WT> P0;
  if constexpr (WLDS) {
    P0 = stage_weights(smem, n.pack, L, L.fwd_total, WT{});
    __syncthreads();
  } else {
    P0 = global_weights(n.pack, L, WT{});
  }
  const int b = blockIdx.x * args.waves + w;
  if (b >= args.B) return;  // wave-uniform; no block barriers after this point
  float* X0 = smem + lds_w + w * Dm::FWD_PERW;
  float* OUT = Dm::QT == 1 ? X0 : X0 + Dm::X0F;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  for (int i = lane; i < Dm::X0F; i += 64) X0[i] = 0.f;
  for (int i = lane; i < 3 * E; i += 64) {
    const int k = i / E, f = i % E;
    X0[(2 * na + k) * Dm::LDX + f] = n.hw0 ? n.hw0[(size_t)b * 3 * E + i] : 0.f;
  }
  MixIn<E, A> in;
  mix_load<E, A>(args, n, b, 0, in, na);
  for (int t = 0; t < n.T; ++t) {
    T2O_MARK(0);
    const Wts<WT> P = step_view(P0);
    // (swizzles per product, as the BPTT kernels: hoisted — 190 VGPRs, 5 % fewer
    // instructions per step — the kernel measured slower, 0.488 -> 0.512 ms,
    // interleaved A/B, profiles/r4_c/)
    mix_keys<E, A>(P, L, in, X0, na);
    const float myq = mix_qv<E, A>(n, in, args.n_actions, args.avail != nullptr);
    __builtin_amdgcn_sched_barrier(0);  // every read of this step's inputs issued before they are reloaded
    if (t + 1 < n.T) mix_load<E, A>(args, n, b, t + 1, in, na);  // prefetch step t+1 (in is consumed)
    wave_sync();
    KeyFrags<E, Dm::KT, sizeof(WT) == 2> K;
    K.template load<Dm::LDX>(X0);
    T2O_MARK(1);
#pragma unroll
    for (int qt = 0; qt < Dm::QT; ++qt) {
      if (RT == 1 && 16 * qt >= nq) break;  // (wave-uniform) query tiles past the real rows
      const int q = 16 * qt + c;
      f4 x[ET];
#pragma unroll
      for (int ft = 0; ft < ET; ++ft)
        x[ft] = q < nq ? ld4(X0 + (na + q) * Dm::LDX + 16 * ft + 4 * g) : zero4();
      wave_sync();  // every X0 read done before OUT (may alias X0) is written
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (d > 0 && n.xmid && q < nq) {
          float* xm = n.xmid + ((((size_t)b * n.T + t) * (D - 1) + d - 1) * nq + q) * E;
#pragma unroll
          for (int ft = 0; ft < ET; ++ft) st4(xm + 16 * ft + 4 * g, x[ft]);
        }
        mixer_block_fwd<E, H, Dm::KT, FF, false>(P, L, d, K, lk, x, nullptr);
        if (qt == 0) T2O_MARK(2 + d);
      }
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) st4(OUT + q * Dm::LDO + 16 * ft + 4 * g, x[ft]);
    }
    wave_sync();
    float qv[A];
    bcast_agents<A>(myq, qv);
    float pre_h, pre2;
    const float y = mixer_head<E, A>(P, L, OUT, qv, pre_h, pre2, na, pf, pb);
    const size_t bt = (size_t)b * n.T + t;
    if (lane == 0) n.y[bt] = y;
    if (n.qv && lane < na) n.qv[bt * na + lane] = myq;
    float hv[(3 * E + 63) / 64];
#pragma unroll
    for (int k = 0; k < (3 * E + 63) / 64; ++k) {
      const int i = lane + 64 * k;
      hv[k] = i < 3 * E ? OUT[(na + i / E) * Dm::LDO + i % E] : 0.f;
      if (i < 3 * E) n.hw[bt * 3 * E + i] = hv[k];
    }
    if (n.xout) {
      for (int i = lane; i < nq * E; i += 64) n.xout[bt * nq * E + i] = OUT[(i / E) * Dm::LDO + i % E];
    }
    wave_sync();  // OUT (may alias X0) fully read before the hyper rows change
#pragma unroll
    for (int k = 0; k < (3 * E + 63) / 64; ++k) {
      const int i = lane + 64 * k;
      if (i < 3 * E) X0[(2 * na + i / E) * Dm::LDX + i % E] = hv[k];
    }
    wave_sync();
    T2O_MARK(2 + D);
    if (blockIdx.y == 0) T2O_PROF_SAVE(t, 2 + D);
  }
}

template <int E, int H, int D, int A, int FF, int RT, typename WT>
int launch_mixer_fwd(const MixerFwdArgs& args, int nnet, hipStream_t stream) {
  if (!kernel_layout_matches<E, H, D, FF, WT>(args.L)) return T2O_EINVAL;  // (kernels use the compile-time offsets)
  using Dm = MixDims<E, A>;
  MixerFwdArgs a = args;
  const size_t wfl = (lds_weight_floats<WT>(args.L, args.L.fwd_total) + 15) / 16 * 16, perw = Dm::FWD_PERW;
  // 8 (two per SIMD at the 512-thread bound's 256 registers) / 4 / 2 waves with LDS
  // weights, else 4 waves reading weights from L2
  const MixLaunch m = mix_pick(wfl, perw, 8, 2, 4, 4);
  if (m.waves < 1) return T2O_EUNSUPPORTED;
  a.waves = m.waves;
  a.wlds = m.wlds;
  const size_t lds = m.lds;
  const bool wide = Dm::QT > 1 && a.waves <= 4 && 2 * lds > 160 * 1024;  // one wave per SIMD
  auto kern = wide ? (a.wlds ? mixer_fwd_kernel<E, H, D, A, FF, RT, true, WT, Dm::QT == 1 ? 512 : 256>
                             : mixer_fwd_kernel<E, H, D, A, FF, RT, false, WT, Dm::QT == 1 ? 512 : 256>)
                   : (a.wlds ? mixer_fwd_kernel<E, H, D, A, FF, RT, true, WT> : mixer_fwd_kernel<E, H, D, A, FF, RT, false, WT>);
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((args.B + a.waves - 1) / a.waves, nnet);
  hipLaunchKernelGGL(kern, grid, dim3(64 * a.waves), lds, stream, a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// BPTT.  One wave per episode; the workgroup shares one LDS copy of the
// forward weights (transposed products via matvec_t) beside each wave's key /
// staging buffers.  Per step t (backwards): rebuild X0 from the stored inputs
// and hyper tokens, run the mixing-head backward on the stored final query
// rows, then per query tile recompute the blocks with cache and
// back-propagate.  Outputs per step: grad wrt the qvals (-> the agent's
// chosen-Q grad) and wrt the agent hidden tokens; the hyper-token grad is
// carried to step t-1.  Weight grads: M/N/W1/W2 operand pairs -> tape records
// (query row x step), contracted by t2o_dwgemm.hpp into slab k; state
// embedding / hyper_b2 grads in registers (lane = feature), flushed once;
// vectors by float atomics into the workgroup's slab.
// RT: as mixer_fwd_kernel's
template <int E, int H, int D, int A, int FF, int RT, bool WLDS, typename WT>
__global__ __launch_bounds__(256) void mixer_bwd_kernel(MixerBwdArgs args) {
  using Dm = MixDims<E, A>;
  constexpr int KM = key_mode<Dm::KT, WT>();
  using Bd = MixBwdDims<E, A, KM>;
  constexpr int ET = E / 16, KT = Dm::KT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const MixerFwdArgs& fa = args.f;
  const MixerNet& n = fa.net[0];
  const t2o_layout& L = fa.L;
  const t2o_layout& G = args.G;
  const int na = RT == 1 ? fa.na : A, nq = na + 3, lk = 2 * na + 3;
  const int w = wave_id();
  float* X0 = smem + args.lds_w + w * Bd::PERW;
  float* X0T = X0 + Dm::X0F;  // (KM 1: the transposed key block)
  float* WORK = X0T + Bd::X0TF;
  float* GOUTB = Bd::GOUT ? WORK : WORK;        // head grads (rows of OUT layout)
  float* stage = WORK + Bd::GOUT;               // staging / gX0 region
  float* gs = args.slabs + (size_t)blockIdx.x * G.grad_total;
  // the forward section of the pack in LDS when it fits
  // beside the per-wave buffers, else read through L2 (large mixers)
  Wts<WT> P0 = WLDS ? stage_weights(smem, n.pack, L, L.fwd_total, WT{})
                    : global_weights(n.pack, L, WT{});
  P0.vol = false;  // (Wts::vol: the one-wave multi-tile BPTT measured slower with volatile reads)
  zero_flushed_regions(gs, G, false);
  __syncthreads();
  const int b = blockIdx.x * args.waves + w;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  using Rec = TapeRec<E, H, FF>;
  // each block's records form one compact stream, (step, episode, query row) in
  // order, read by the contraction as 16-record tiles (t2o_bwd_tape_tiles); the
  // last tile's records past the stream's end are zeros
  const size_t nrec = (size_t)fa.B * n.T * nq, ctiles = (nrec + 15) / 16;
  if (blockIdx.x == 0 && w == 0) {
    const int tail = (int)(ctiles * 16 - nrec) * Rec::SIZE;  // elements
    for (int d = 0; d < D; ++d) {
      WT* z = static_cast<WT*>(args.tape) + ((size_t)d * ctiles * 16 + nrec) * Rec::SIZE;
      for (int i = lane_c() + 16 * lane_g(); i < tail; i += 64) z[i] = WT(0.f);
    }
  }
  const int f = lane < E ? lane : 0;
  const bool fv = lane < E;
  // state embedding grads as MFMA tiles: lane (g, c) reg r = dWe[16ft+4g+r][c]
  // (column Fs = d be); hyper_b2 grads per lane (feature)
  f4 gWe[ET];
#pragma unroll
  for (int ft = 0; ft < ET; ++ft) gWe[ft] = zero4();
  f4 ln2[D][2 * ET];  // LN2 vector grads, per-lane partial sums over the episode's steps
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int t = 0; t < 2 * ET; ++t) ln2[d][t] = zero4();
  float gWo = 0.f, gbo = 0.f;
  if (b < fa.B) {
    for (int i = lane; i < Dm::X0F; i += 64) X0[i] = 0.f;
    float ghw[3] = {0.f, 0.f, 0.f};  // grad wrt this step's hyper outputs, lane = feature
    // Multi-tile mixers (A+3 > 16 query rows) hold a register file's worth of
    // state per step: they use the lean block cache (the forward recompute writes
    // the record's X / Z / Y fields itself) and load each step's inputs when the
    // step starts instead of double-buffering them a step ahead — without both,
    // the 16-AGV kernel spilled ~100 registers to scratch.
    constexpr bool LEAN = Dm::QT > 1;
    MixBwdIn<E, A, D> cur, nxt;
    if constexpr (!LEAN) mixb_load<E, A, D>(args, n, b, n.T - 1, cur, na);
    for (int t = n.T - 1; t >= 0; --t) {
      const Wts<WT> P = step_view(P0);
      const size_t bt = (size_t)b * n.T + t;
      if constexpr (LEAN) mixb_load<E, A, D, false>(args, n, b, t, cur, na);  // (block inputs: per tile, below)
      mix_keys<E, A>(P, L, cur.m, X0, na);
#pragma unroll
      for (int k = 0; k < MixBwdIn<E, A, D>::HW; ++k) {
        const int i = lane + 64 * k;
        if (i < 3 * E) X0[(2 * na + i / E) * Dm::LDX + i % E] = cur.hwp[k];
      }
      float* OUT = stage;  // forward final query rows
#pragma unroll
      for (int k = 0; k < MixBwdIn<E, A, D>::XO; ++k) {
        const int i = lane + 64 * k;
        if (i < nq * E) OUT[(i / E) * Bd::LDB + i % E] = cur.xo[k];
      }
      if constexpr (!LEAN) {
        if (t > 0) mixb_load<E, A, D>(args, n, b, t - 1, nxt, na);  // prefetch step t-1
      }
      wave_sync();
      // ---- mixing head backward (lanes = features)
#pragma unroll
      for (int k = 0; k < 3; ++k) ghw[k] += cur.ghx[k];
      float* GOUT = Bd::GOUT ? GOUTB : stage;
      mixer_head_bwd<E, A, WT, Bd::LDB>(P, L, OUT, GOUT, cur.m.qs[0], cur.gy, ghw, args.gqv + bt * na + lane, gWo, gbo, na,
                           RT ? L.pos_func : T2O_POS_ABS, RT ? L.pos_beta : 1.f);
      for (int i = nq * Bd::LDB + lane; i < Bd::OUTB; i += 64) GOUT[i] = 0.f;
      wave_sync();
      // ---- blocks backward per query tile; gX0 accumulates in registers
      KeyFrags<E, KT, sizeof(WT) == 2, KM> K;
      load_keys<Dm::LDX>(K, X0, X0T);
      f4 gX0[KT][ET];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) gX0[kt][ft] = zero4();
      f4 gq0[LEAN ? 1 : Dm::QT][ET];
      if constexpr (LEAN) {
        // one query tile at a time, not unrolled: its grads come from and go back
        // to GOUT (LDS), its block inputs straight from HBM
        const int nqt = (nq + 15) / 16;
#pragma unroll 1
        for (int qt = 0; qt < nqt; ++qt) {
        const Wts<WT> Pq = step_view(P);  // (opaque per query tile: weight reads stay in the loop)
          const int q = 16 * qt + c;
          f4 gx[ET];
#pragma unroll
          for (int ft = 0; ft < ET; ++ft) gx[ft] = ld4(GOUT + (16 * qt + c) * Bd::LDB + 16 * ft + 4 * g);
#pragma unroll
          for (int d = D - 1; d >= 0; --d) {
            f4 x[ET];
#pragma unroll
            for (int ft = 0; ft < ET; ++ft) x[ft] = q < nq ? ld4(X0 + (na + q) * Dm::LDX + 16 * ft + 4 * g) : zero4();
            if (d > 0) {
              if (args.xmid) {
#pragma unroll
                for (int ft = 0; ft < ET; ++ft)
                  x[ft] = q < nq ? ld4(args.xmid + ((bt * (D - 1) + d - 1) * nq + q) * E + 16 * ft + 4 * g)
                                 : zero4();
              } else {
                for (int dd = 0; dd < d; ++dd) mixer_block_fwd<E, H, KT, FF, false>(Pq, L, dd, K, lk, x, nullptr);
              }
            }
            // a tile's 16 records, or the nq - 16·qt real ones of the last
            WT* tile = static_cast<WT*>(args.tape) +
                       ((size_t)d * ctiles * 16 + ((size_t)t * fa.B + b) * nq + 16 * qt) * Rec::SIZE;
            MixerCacheLean<E, H, KT, FF> cache;
            const MaskedRec<WT, 2> rec(tile, min(16, nq - 16 * qt), Rec::SIZE);  // non-temporal (MaskedRec)
            mixer_block_fwd_lean<E, H, KT, FF>(Pq, L, d, K, lk, x, cache, rec);
            mixer_block_bwd_lean<E, H, KT, FF>(Pq, L, gs, rec, stage, d, K, lk, gX0, cache, gx, ln2[d]);
          }
          wave_sync();
#pragma unroll
          for (int ft = 0; ft < ET; ++ft)
            st4(GOUT + (16 * qt + c) * Bd::LDB + 16 * ft + 4 * g, q < nq ? gx[ft] : zero4());
        }
      } else {
      static_assert(LEAN || Dm::QT == 1, "the unrolled path runs one query tile");
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) gq0[0][ft] = ld4(GOUT + c * Bd::LDB + 16 * ft + 4 * g);
      wave_sync();
      {
        const int q = c;
        f4 gx[ET];
        f4 xs[D][ET];
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) {
          gx[ft] = gq0[0][ft];
          xs[0][ft] = q < nq ? ld4(X0 + (na + q) * Dm::LDX + 16 * ft + 4 * g) : zero4();
        }
        if (args.xmid) {  // stored block inputs of blocks 1..D-1 (no plain recompute)
#pragma unroll
          for (int d = 1; d < D; ++d)
#pragma unroll
            for (int ft = 0; ft < ET; ++ft) xs[d][ft] = cur.xm[0][d - 1][ft];
        } else {
#pragma unroll
          for (int d = 0; d + 1 < D; ++d) {
            f4 x[ET];
#pragma unroll
            for (int ft = 0; ft < ET; ++ft) x[ft] = xs[d][ft];
            mixer_block_fwd<E, H, KT, FF, false>(P, L, d, K, lk, x, nullptr);
#pragma unroll
            for (int ft = 0; ft < ET; ++ft) xs[d + 1][ft] = x[ft];
          }
        }
#pragma unroll
        for (int d = D - 1; d >= 0; --d) {
          f4 x[ET];
#pragma unroll
          for (int ft = 0; ft < ET; ++ft) x[ft] = xs[d][ft];
          // the (episode, step)'s nq records of the block's compact stream
          WT* tile = static_cast<WT*>(args.tape) + ((size_t)d * ctiles * 16 + ((size_t)t * fa.B + b) * nq) * Rec::SIZE;
          MixerCache<E, H, KT, FF> cache;
          mixer_block_fwd<E, H, KT, FF, true>(P, L, d, K, lk, x, &cache);
          mixer_block_bwd<E, H, KT, FF>(P, L, G, gs, c < nq ? tile : nullptr, stage, d, K, gX0, cache, gx, ln2[d]);
        }
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) gq0[0][ft] = q < nq ? gx[ft] : zero4();
      }
      }
      // ---- state embedding grads straight from the key-grad registers:
      // dWe[f][fs] (+ d be[f] in column Fs) += Σ_{entity j} gX0[j][f] · [s_j, 1][fs]
#pragma unroll
      for (int s = 0; s < Dm::ST; ++s)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) {
          f4 am;
#pragma unroll
          for (int r = 0; r < 4; ++r) am[r] = 16 * s + 4 * g + r < na ? gX0[s][ft][r] : 0.f;
          if constexpr (sizeof(WT) == 2) {
            gWe[ft] = mfma_b16(to_bf4(am), to_bf4(cur.stT[s]), gWe[ft]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) gWe[ft] = mfma4(am[r], cur.stT[s][r], gWe[ft]);
          }
        }
      wave_sync();
      // ---- gX0 registers -> LDS rows [key][feature], plus the query path
      float* GX0 = stage;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft)
#pragma unroll
          for (int r = 0; r < 4; ++r) GX0[(16 * kt + 4 * g + r) * Bd::LDB + 16 * ft + c] = gX0[kt][ft][r];
      wave_sync();
#pragma unroll
      for (int qt = 0; qt < Dm::QT; ++qt) {
        const int q = 16 * qt + c;
        if (q < nq) {
#pragma unroll
          for (int ft = 0; ft < ET; ++ft) {
            float* dst = GX0 + (na + q) * Bd::LDB + 16 * ft + 4 * g;
            const f4 gq = LEAN ? ld4(GOUT + q * Bd::LDB + 16 * ft + 4 * g) : gq0[0][ft];
            st4(dst, ld4(dst) + gq);
          }
        }
      }
      wave_sync();
      // ---- key-token grads: agent hidden tokens out, hyper tokens carried
      for (int i = lane; i < na * E / 4; i += 64)
        st4(args.ghid + bt * na * E + 4 * i, ld4(GX0 + (na + 4 * i / E) * Bd::LDB + (4 * i) % E));
#pragma unroll
      for (int k = 0; k < 3; ++k) ghw[k] = fv ? GX0[(2 * na + k) * Bd::LDB + f] : 0.f;
      wave_sync();
      if constexpr (!LEAN) cur = nxt;
    }
    if (args.ghw0 && fv) {
#pragma unroll
      for (int k = 0; k < 3; ++k) args.ghw0[((size_t)b * 3 + k) * E + f] = ghw[k];
    }
  }
  flush_in_wave_order([&] {
    if (b < fa.B) {
#pragma unroll
      for (int ft = 0; ft < ET; ++ft)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int fe = 16 * ft + 4 * g + r;
          if (c < fa.Fs) unsafeAtomicAdd(gs + G.We + fe * 16 + c, gWe[ft][r]);
          else if (c == fa.Fs) unsafeAtomicAdd(gs + G.be + fe, gWe[ft][r]);
        }
      if (fv) unsafeAtomicAdd(gs + G.Wo + f, gWo);
      if (lane == 0) unsafeAtomicAdd(gs + G.bo, gbo);
      ln2_flush<E, D>(gs, G, ln2);
    }
  });
}

// ---- two waves per episode (depth 2, one query tile) ------------------------
// As the agent's pipelined BPTT (t2o_agent.hip, agent_bwd_pipe_kernel): each
// wave of a pair owns one transformer block of one episode, and the two
// interleave so that one's recompute overlaps the other's backward (phases
// separated by the pair's barrier, t2o_common.hpp PairBarrier):
//   block-1 wave: keys+fwd1(T-1) | head+bwd1(T-1) | keys+fwd1(T-2) | head+bwd1(T-2) | ...
//   block-0 wave:        -       |   fwd0(T-1)    |  bwd0+X0(T-1)  |   fwd0(T-2)    | ...
// The dependent chain per step is head -> bwd1 -> bwd0 -> hyper-token grads ->
// head of the step before; the recomputes (key block, block forwards with
// cache) come off it.  Pair LDS: the key block X0 (written by the block-1
// wave's recompute, read by both recomputes, untouched in backward phases) and
// one region R owned by whichever wave is in its backward phase: head rows and
// dW staging, then the hand-over 1 -> 0 [block-1 key grads (rows < LK) | grad
// wrt the block-1 input (query rows, in R's padding rows)], then the step's
// total key grads written by the block-0 wave, whose hyper rows the block-1
// wave reads at its next backward.  Per-step math, records and slab sums are
// those of mixer_bwd_kernel; the block cache is the lean one (MixerCacheLean)
// so that a wave fits half a register file (two waves per SIMD), and records
// are written through MaskedRec (tape tiles of exactly the Q query rows).
template <int E, int A>
struct MixPipeDims {
  using Dm = MixDims<E, A>;
  using Bd = MixBwdDims<E, A>;
// Row stride of the pair region's [row][feature] blocks.  E + 4 (the other
// kernels' LDO) removes their T-layout bank conflicts here too, but measured slower
// in this register-bound kernel: interleaved A/B, overlapped, 3 rounds
// (profiles/r3_ab2/): mixer_bwd 0.618 ms at E vs 0.630 at E + 4.
  static constexpr int LDR = E;
  static constexpr int XCH = Dm::LKCAP * LDR;  // offset of the query-row grads in R
  static constexpr int R0 = Bd::W0 > Dm::KT * 16 * LDR ? Bd::W0 : Dm::KT * 16 * LDR;
  // (the hand-over needs R to hold the key grads and, past them, the query-row grads)
  static constexpr int REGION = R0 > XCH + Dm::QCAP * LDR ? R0 : XCH + Dm::QCAP * LDR;
  static constexpr int PAIRF = Dm::X0F + REGION;
  static constexpr bool OK = Dm::QT == 1;
};

// T2O_MIXER_BWD=single selects the one-wave kernel (A/B timing, parity cross-check)
inline bool mixer_bwd_single_wave() {
  static const bool single = [] {
    const char* e = getenv("T2O_MIXER_BWD");
    return e && e[0] == 's';
  }();
  return single;
}

// The block-1 wave's per-step inputs (none recurrent), loaded at the start of
// its recompute phase (which has slack under the block-0 backward) and held
// through its backward phase; the backward's Q selection is qmode 0, so only
// qvals ride along.
template <int E, int A>
struct MixPIn {
  using Dm = MixDims<E, A>;
  static constexpr int ET = E / 16;
  static constexpr int HV = MixIn<E, A>::HV, HW = MixBwdIn<E, A, 2>::HW, XO = MixBwdIn<E, A, 2>::XO;
  f4 st[Dm::ST];
  f4 hid[HV];
  float qv;
  float hwp[HW];
  float xo[XO];
  float ghx[3];
  float gy;
  f4 xm[ET];  // stored block-1 input (T-layout query rows)
};

template <int E, int A>
T2O_DEV void mixp_load(const MixerBwdArgs& args, int b, int t, MixPIn<E, A>& in, int na) {
  using Dm = MixDims<E, A>;
  using In = MixPIn<E, A>;
  const MixerFwdArgs& fa = args.f;
  const MixerNet& n = fa.net[0];
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  const int nq = na + 3;
  const float* st = fa.states + b * fa.st_sb + t * fa.st_st;
#pragma unroll
  for (int s = 0; s < Dm::ST; ++s) {
    const int j = 16 * s + c;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * g + r;
      in.st[s][r] = ld_or0(st, j * fa.Fs + f, j < na && f < fa.Fs);
    }
  }
  const float* hd = n.hid + b * n.hid_sb + t * n.hid_st;
#pragma unroll
  for (int k = 0; k < In::HV; ++k) {
    const int i = lane + 64 * k;
    in.hid[k] = i < na * E / 4 ? ld4(hd + 4 * i) : zero4();
  }
  const size_t bt = (size_t)b * n.T + t;
  in.qv = n.qv_in[bt * na + (lane < na ? lane : na - 1)];
#pragma unroll
  for (int k = 0; k < In::HW; ++k) {
    const int i = lane + 64 * k;
    float v = 0.f;
    if (i < 3 * E) v = t > 0 ? args.hw[(bt - 1) * 3 * E + i] : (n.hw0 ? n.hw0[(size_t)b * 3 * E + i] : 0.f);
    in.hwp[k] = v;
  }
#pragma unroll
  for (int k = 0; k < In::XO; ++k) {
    const int i = lane + 64 * k;
    in.xo[k] = i < nq * E ? args.xout[bt * nq * E + i] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) in.ghx[k] = (args.ghw_ext && lane < E) ? args.ghw_ext[(bt * 3 + k) * E + lane] : 0.f;
  in.gy = args.gy[bt];
#pragma unroll
  for (int ft = 0; ft < In::ET; ++ft)
    in.xm[ft] = c < nq ? ld4(args.xmid + (bt * nq + c) * E + 16 * ft + 4 * g) : zero4();
}

template <int E, int A>
T2O_DEV void mixp_load_stT(const MixerFwdArgs& fa, int b, int t, f4 (&stT)[MixDims<E, A>::ST], int na) {
  using Dm = MixDims<E, A>;
  const int c = lane_c(), g = lane_g();
  const float* st = fa.states + b * fa.st_sb + t * fa.st_st;
#pragma unroll
  for (int s = 0; s < Dm::ST; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * s + 4 * g + r;
      float v = ld_or0(st, j * fa.Fs + c, j < na && c < fa.Fs);
      if (j < na && c == fa.Fs) v = 1.f;
      stT[s][r] = v;
    }
}

// block-1 wave: key block + block-1 recompute, then head + block-1 backward
template <int E, int H, int A, int FF, typename WT>
T2O_DEV void mixp_block1(const MixerBwdArgs& args, const Wts<WT>& P0, const t2o_layout& L, const t2o_layout& G,
                         float* __restrict__ gs, float* X0, float* R, int b, PairBarrier& pbar, int na, int pf,
                         float pb) {
  const t2o_layout Lb = block_view(L, 1), Gb = block_view(G, 1);  // (constant block: immediate offsets)
  using Dm = MixDims<E, A>;
  using Pd = MixPipeDims<E, A>;
  using In = MixPIn<E, A>;
  using Rec = TapeRec<E, H, FF>;
  constexpr int ET = E / 16, KT = Dm::KT;
  constexpr bool BF = sizeof(WT) == 2;
  const MixerFwdArgs& fa = args.f;
  const MixerNet& n = fa.net[0];
  const int T = n.T;
  const int nq = na + 3, lk = 2 * na + 3;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  const int f = lane < E ? lane : 0;
  const bool fv = lane < E;
  // block 1's compact record stream (mixer_bwd_kernel)
  const size_t ctiles = ((size_t)fa.B * T * nq + 15) / 16;
  constexpr size_t RECD = 1;  // tape block
  f4 ln2[2 * ET];
#pragma unroll
  for (int i = 0; i < 2 * ET; ++i) ln2[i] = zero4();
  float gWo = 0.f, gbo = 0.f;
  In cur;
  for (int t = T - 1; t >= 0; --t) {
    const size_t bt = (size_t)b * T + t;
    // the (episode, step)'s nq records
    const MaskedRec<WT> rec(static_cast<WT*>(args.tape) + (RECD * ctiles * 16 + ((size_t)t * fa.B + b) * nq) * Rec::SIZE,
                            nq, Rec::SIZE);
    MixerCacheLean<E, H, KT, FF> cache;
    KeyFrags<E, KT, BF> K;
    {  // ---- recompute: key block of step t, block-1 forward with cache
      // (this phase has slack under the block-0 backward: the step's inputs load here)
      mixp_load<E, A>(args, b, t, cur, na);
      const Wts<WT> P = step_view(P0);
      mix_keys<E, A>(P, L, cur, X0, na);
#pragma unroll
      for (int k = 0; k < In::HW; ++k) {
        const int i = lane + 64 * k;
        if (i < 3 * E) X0[(2 * na + i / E) * Dm::LDX + i % E] = cur.hwp[k];
      }
      wave_sync();
      K.template load<Dm::LDX>(X0);
      f4 x[ET];
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) x[ft] = cur.xm[ft];
      mixer_block_fwd_lean<E, H, KT, FF>(P, Lb, 0, K, lk, x, cache, rec);
    }
    pbar.sync();
    {  // ---- backward: mixing head, block 1
      const Wts<WT> P = step_view(P0);
      float ghw[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) ghw[k] = (t < T - 1 && fv) ? R[(2 * na + k) * Pd::LDR + f] : 0.f;
      wave_sync();
      float* OUT = R;  // forward final query rows, then their grads in place
#pragma unroll
      for (int k = 0; k < In::XO; ++k) {
        const int i = lane + 64 * k;
        if (i < nq * E) OUT[(i / E) * Pd::LDR + i % E] = cur.xo[k];
      }
      wave_sync();
#pragma unroll
      for (int k = 0; k < 3; ++k) ghw[k] += cur.ghx[k];
      mixer_head_bwd<E, A, WT, Pd::LDR>(P, L, OUT, OUT, cur.qv, cur.gy, ghw, args.gqv + bt * na + lane, gWo, gbo, na,
                                        pf, pb);
      wave_sync();
      f4 gx[ET];
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) gx[ft] = c < nq ? ld4(OUT + c * Pd::LDR + 16 * ft + 4 * g) : zero4();
      wave_sync();
      f4 gX0[KT][ET];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) gX0[kt][ft] = zero4();
      mixer_block_bwd_lean<E, H, KT, FF>(P, Lb, gs, rec, R, 0, K, lk, gX0, cache, gx, ln2);
      wave_sync();
      // hand-over to the block-0 wave
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * kt + 4 * g + r;
            if (row < lk) R[row * Pd::LDR + 16 * ft + c] = gX0[kt][ft][r];
          }
      if (c < nq) {
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) st4(R + Pd::XCH + c * Pd::LDR + 16 * ft + 4 * g, gx[ft]);
      }
    }
    pbar.sync();
  }
  pbar.sync();  // the block-0 wave's last backward phase
  flush_in_wave_order([&] {
    vec_accumulate_g<ET>(gs + Gb.g2[0], &ln2[0]);
    vec_accumulate_g<ET>(gs + Gb.n2[0], &ln2[ET]);
    if (fv) unsafeAtomicAdd(gs + Gb.Wo + f, gWo);
    if (lane == 0) unsafeAtomicAdd(gs + Gb.bo, gbo);
  });
}

// block-0 wave: block-0 recompute, then block-0 backward and the step's key grads
template <int E, int H, int A, int FF, typename WT>
T2O_DEV void mixp_block0(const MixerBwdArgs& args, const Wts<WT>& P0, const t2o_layout& L, const t2o_layout& G,
                         float* __restrict__ gs, const float* X0, float* R, int b, PairBarrier& pb, int na) {
  const t2o_layout Lb = block_view(L, 0), Gb = block_view(G, 0);
  using Dm = MixDims<E, A>;
  using Pd = MixPipeDims<E, A>;
  using Rec = TapeRec<E, H, FF>;
  constexpr int ET = E / 16, KT = Dm::KT;
  constexpr bool BF = sizeof(WT) == 2;
  const MixerFwdArgs& fa = args.f;
  const int T = fa.net[0].T;
  const int nq = na + 3, lk = 2 * na + 3;
  const size_t ctiles = ((size_t)fa.B * T * nq + 15) / 16;
  constexpr size_t RECD = 0;  // tape block
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  const int f = lane < E ? lane : 0;
  const bool fv = lane < E;
  f4 ln2[2 * ET], gWe[ET];
#pragma unroll
  for (int i = 0; i < ET; ++i) ln2[i] = ln2[ET + i] = gWe[i] = zero4();
  f4 stT[Dm::ST];
  pb.sync();  // one phase behind the block-1 wave
  for (int t = T - 1; t >= 0; --t) {
    const size_t bt = (size_t)b * T + t;
    // the (episode, step)'s nq records
    const MaskedRec<WT> rec(static_cast<WT*>(args.tape) + (RECD * ctiles * 16 + ((size_t)t * fa.B + b) * nq) * Rec::SIZE,
                            nq, Rec::SIZE);
    MixerCacheLean<E, H, KT, FF> cache;
    KeyFrags<E, KT, BF> K;
    {  // ---- recompute: block-0 forward with cache (queries = X0's last na+3 rows)
      mixp_load_stT<E, A>(fa, b, t, stT, na);  // for this step's state-embedding grads
      const Wts<WT> P = step_view(P0);
      K.template load<Dm::LDX>(X0);
      f4 x[ET];
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) x[ft] = c < nq ? ld4(X0 + (na + c) * Dm::LDX + 16 * ft + 4 * g) : zero4();
      mixer_block_fwd_lean<E, H, KT, FF>(P, Lb, 0, K, lk, x, cache, rec);
    }
    pb.sync();
    {  // ---- backward: block 0, then the step's key-token grads
      const Wts<WT> P = step_view(P0);
      f4 gX0[KT][ET], gx[ET];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * kt + 4 * g + r;
            gX0[kt][ft][r] = row < lk ? R[row * Pd::LDR + 16 * ft + c] : 0.f;
          }
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) gx[ft] = c < nq ? ld4(R + Pd::XCH + c * Pd::LDR + 16 * ft + 4 * g) : zero4();
      wave_sync();
      mixer_block_bwd_lean<E, H, KT, FF>(P, Lb, gs, rec, R, 0, K, lk, gX0, cache, gx, ln2);
      // state embedding grads from the key-grad registers (as mixer_bwd_kernel)
#pragma unroll
      for (int s = 0; s < Dm::ST; ++s)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) {
          f4 am;
#pragma unroll
          for (int r = 0; r < 4; ++r) am[r] = 16 * s + 4 * g + r < na ? gX0[s][ft][r] : 0.f;
          if constexpr (BF) {
            gWe[ft] = mfma_b16(to_bf4(am), to_bf4(stT[s]), gWe[ft]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) gWe[ft] = mfma4(am[r], stT[s][r], gWe[ft]);
          }
        }
      wave_sync();
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft)
#pragma unroll
          for (int r = 0; r < 4; ++r) R[(16 * kt + 4 * g + r) * Pd::LDR + 16 * ft + c] = gX0[kt][ft][r];
      wave_sync();
      if (c < nq) {  // the query path: block-0 input rows are X0's last na+3 rows
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) {
          float* dst = R + (na + c) * Pd::LDR + 16 * ft + 4 * g;
          st4(dst, ld4(dst) + gx[ft]);
        }
      }
      wave_sync();
      for (int i = lane; i < na * E / 4; i += 64)
        st4(args.ghid + bt * na * E + 4 * i, ld4(R + (na + 4 * i / E) * Pd::LDR + (4 * i) % E));
      if (t == 0 && args.ghw0 && fv) {
#pragma unroll
        for (int k = 0; k < 3; ++k) args.ghw0[((size_t)b * 3 + k) * E + f] = R[(2 * na + k) * Pd::LDR + f];
      }
    }
    pb.sync();
  }
  flush_in_wave_order([&] {
#pragma unroll
    for (int ft = 0; ft < ET; ++ft)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int fe = 16 * ft + 4 * g + r;
        if (c < fa.Fs) unsafeAtomicAdd(gs + Gb.We + fe * 16 + c, gWe[ft][r]);
        else if (c == fa.Fs) unsafeAtomicAdd(gs + Gb.be + fe, gWe[ft][r]);
      }
    vec_accumulate_g<ET>(gs + Gb.g2[0], &ln2[0]);
    vec_accumulate_g<ET>(gs + Gb.n2[0], &ln2[ET]);
  });
  (void)fv;
}

template <typename WT>
inline __host__ __device__ int64_t mixp_weight_elems(const t2o_layout& L) {
  return sizeof(WT) == 4 ? L.fwd_total : L.total;
}

template <int E, int H, int D, int A, int FF, int RT, typename WT>
T2O_DEV void mixer_bwd_pipe_body(const MixerBwdArgs& args, const t2o_layout& L, const t2o_layout& G) {
  static_assert(D == 2 && MixPipeDims<E, A>::OK, "one wave per block of a depth-2 stack, one query tile");
  using Dm = MixDims<E, A>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const int na = RT == 1 ? args.f.na : A;
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  // the block this wave owns.  Waves w and w + 4 share a SIMD: with four pairs,
  // pairs 2-3 swap their block roles so every SIMD holds one block-0 and one
  // block-1 wave (the two phases of a barrier interval differ in cost)
#ifndef T2O_PIPE_NO_SIMD_MIX
  const int d = (w ^ (w >> 2)) & 1;
#else
  const int d = w & 1;
#endif
  const int pr = w >> 1; // the episode within the workgroup
  float* X0 = smem + args.lds_w + pr * MixPipeDims<E, A>::PAIRF;
  float* R = X0 + Dm::X0F;
  float* gs = args.slabs + (size_t)blockIdx.x * G.grad_total;
  // bf16: with the transposed copies (the pipelined kernel is register-bound at two
  // waves per SIMD; transposed reads of the forward image cost it spills)
  const Wts<WT> P0 = stage_weights(smem, args.f.net[0].pack, L, mixp_weight_elems<WT>(L), WT{}, false);
  zero_flushed_regions(gs, G, false);
  if (d == 1)
    for (int i = threadIdx.x & 63; i < Dm::X0F; i += 64) X0[i] = 0.f;
  int* const flags = reinterpret_cast<int*>(smem + args.lds_w + args.waves * MixPipeDims<E, A>::PAIRF);
  if (threadIdx.x < PAIR_FLAG_FLOATS) flags[threadIdx.x] = 0;
  if (blockIdx.x == 0 && threadIdx.x < 64) {  // zero each block's compact stream past its last record
    using Rec = TapeRec<E, H, FF>;
    const size_t nrec = (size_t)args.f.B * args.f.net[0].T * (na + 3), ctiles = (nrec + 15) / 16;
    const int tail = (int)(ctiles * 16 - nrec) * Rec::SIZE;
    for (int dd = 0; dd < D; ++dd) {
      WT* z = static_cast<WT*>(args.tape) + ((size_t)dd * ctiles * 16 + nrec) * Rec::SIZE;
      for (int i = threadIdx.x; i < tail; i += 64) z[i] = WT(0.f);
    }
  }
  __syncthreads();
  PairBarrier pb = PairBarrier::make(flags, w);  // partner: the pair's other wave
  const int b = blockIdx.x * args.waves + pr;  // the launcher makes every pair valid
  // the block-1 wave issues first on its SIMD.  With pair barriers (each pair
  // waits only for itself) that is the head + bwd1 end of the dependent chain:
  // A/B, overlapped, 3 rounds: block 1 mixer_bwd 0.596 ms / update 2.556 ms,
  // block 0 0.634 / 2.602, none 0.637 / 2.586 (profiles/r2_pb/r2_prio_ovl/).
  // (Under workgroup barriers block 0 had measured better: 0.654 vs 0.665.)
  if (d == 1) __builtin_amdgcn_s_setprio(1);  // the block-1 waves issue first on their SIMD
  if (d == 1)
    mixp_block1<E, H, A, FF, WT>(args, P0, L, G, gs, X0, R, b, pb, na, RT ? L.pos_func : T2O_POS_ABS,
                                 RT ? L.pos_beta : 1.f);
  else mixp_block0<E, H, A, FF, WT>(args, P0, L, G, gs, X0, R, b, pb, na);
}

// bf16: the pack / gradient offsets as compile-time constants (t2o_layout.hpp
// kernel_layout): SGPR spills (to VGPR lanes, a v_readlane per reload in the
// step loop) 169 -> 113, mixer_bwd 0.598 -> 0.582 ms, update 2.490 -> 2.483 ms
// (interleaved A/B, overlapped, 3 rounds, profiles/r3_ab5/).  fp32 keeps the
// kernel-argument layout: with constants its VGPR spills rose 5 -> 88 and the
// kernel 1.74 -> 2.14 ms (profiles/r3_ab4f/); the other kernels measured no
// gain with them (agent_fwd +2 %, profiles/r3_ab4/).
template <int E, int H, int D, int A, int FF, int RT, typename WT>
__global__ __launch_bounds__(512) void mixer_bwd_pipe_kernel(MixerBwdArgs args) {
  if constexpr (sizeof(WT) == 2)
    mixer_bwd_pipe_body<E, H, D, A, FF, RT, WT>(args, kernel_layout<E, H, D, FF, WT>(args.f.L),
                                                kernel_grad_layout<E, H, D, FF, WT>());
  else
    mixer_bwd_pipe_body<E, H, D, A, FF, RT, WT>(args, args.f.L, args.G);
}

template <int E, int H, int D, int A, int FF, int RT, typename WT>
int launch_mixer_bwd(MixerBwdArgs& args, int max_slabs, int* nslab, hipStream_t stream) {
  if (!kernel_layout_matches<E, H, D, FF, WT>(args.f.L)) return T2O_EINVAL;  // (compile-time offsets)
  constexpr int PERW = MixBwdDims<E, A, key_mode<MixDims<E, A>::KT, WT>()>::PERW;
  const t2o_layout& L = args.f.L;
  args.lds_w = (int)((lds_weight_floats<WT>(L, L.fwd_total) + 15) / 16 * 16);
  if constexpr (D == 2 && MixPipeDims<E, A>::OK) {
    if (args.xmid && !mixer_bwd_single_wave()) {
      const int lds_w = (int)((lds_weight_floats<WT>(L, mixp_weight_elems<WT>(L)) + 15) / 16 * 16);
      for (int pairs = 4; pairs >= 1; pairs >>= 1) {
        const size_t lds =
            sizeof(float) * ((size_t)lds_w + (size_t)pairs * MixPipeDims<E, A>::PAIRF + PAIR_FLAG_FLOATS);
        if (lds > 160 * 1024 || args.f.B % pairs) continue;
        args.waves = pairs;
        args.lds_w = lds_w;
        const int grid = args.f.B / pairs;
        if (grid > max_slabs) return T2O_EINVAL;
        auto kern = mixer_bwd_pipe_kernel<E, H, D, A, FF, RT, WT>;
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(128 * pairs), lds, stream, args);
        *nslab = grid;
        return (int)hipGetLastError();
      }
    }
  }
  // up to 4 waves (launch bound 256; the kernel takes the whole register file)
  const MixLaunch m = mix_pick((size_t)args.lds_w, PERW, 4, 1, 4, 1);
  if (m.waves < 1) return T2O_EUNSUPPORTED;
  args.waves = m.waves;
  const bool wlds = m.wlds;
  if (!wlds) args.lds_w = 0;
  const size_t lds = m.lds;
  const int grid = (args.f.B + args.waves - 1) / args.waves;
  if (grid > max_slabs) return T2O_EINVAL;
  auto kern = wlds ? mixer_bwd_kernel<E, H, D, A, FF, RT, true, WT> : mixer_bwd_kernel<E, H, D, A, FF, RT, false, WT>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * args.waves), lds, stream, args);
  *nslab = grid;
  return (int)hipGetLastError();
}

}  // namespace

// diagnostic builds only (-DT2O_PHASE_PROF, tools/phase_prof.py)
T2O_PROF_READER(t2o_prof_read_mixer)

static int mixer_fwd_impl(const t2o_layout* L, const float* pack_on, const float* pack_tg,
                          const float* states, int64_t st_sb, int64_t st_st,
                          const float* hid_on, const float* hid_tg, int64_t hid_sb, int64_t hid_st,
                          const float* hw0_on, const float* hw0_tg, int qmode_on, int qmode_tg,
                          const float* qv_on, const float* qv_tg, const float* q_on,
                          const float* q_tg, int q_ts, int n_actions, const int64_t* actions,
                          int64_t act_sb, int64_t act_st, const int32_t* avail, int64_t av_sb,
                          int64_t av_st, float* y_on, float* hw_on, float* qvo_on, float* xout_on,
                          float* xmid_on, float* y_tg, float* hw_tg, float* qvo_tg, float* xout_tg,
                          float* xmid_tg, int B, int T_on, int T_tg, int phase, int t0, int t1, void* stream) {
  if (!L || L->kind != 1 || !pack_on || !states || !hid_on || !y_on || !hw_on || B < 1 || T_on < 1 ||
      L->E > 64)
    return T2O_EINVAL;
  if (phase && (L->generic || !t2o::mixer_split_taken(*L, B))) return T2O_EUNSUPPORTED;
  if (L->generic) {
    auto ok = [&](int mode, const float* qv, const float* qsel) {
      return mode == 0 ? qv != nullptr : mode == 1 ? (qsel && actions) : mode == 2 ? (qsel && q_on) : false;
    };
    if (!ok(qmode_on, qv_on, q_on) || (pack_tg && (!hid_tg || !y_tg || !hw_tg || T_tg < 1 || !ok(qmode_tg, qv_tg, q_tg))))
      return T2O_EINVAL;
    return gen_mixer_unroll_fwd(L, pack_on, pack_tg, states, st_sb, st_st, hid_on, hid_tg, hid_sb, hid_st, hw0_on,
                                hw0_tg, qmode_on, qmode_tg, qv_on, qv_tg, q_on, q_tg, q_ts, n_actions, actions,
                                act_sb, act_st, avail, av_sb, av_st, y_on, hw_on, qvo_on, xout_on, xmid_on, y_tg,
                                hw_tg, qvo_tg, xout_tg, xmid_tg, B, T_on, T_tg, (hipStream_t)stream);
  }
  MixerFwdArgs a{};
  a.L = *L;
  a.states = states;
  a.st_sb = st_sb;
  a.st_st = st_st;
  a.qarg = q_on;
  a.q_ts = q_ts;
  a.n_actions = n_actions;
  a.actions = actions;
  a.act_sb = act_sb;
  a.act_st = act_st;
  a.avail = avail;
  a.av_sb = av_sb;
  a.av_st = av_st;
  a.B = B;
  a.Fs = L->F;
  a.na = L->n_ent;
  auto check_mode = [&](int mode, const float* qv, const float* qsel) {
    if (mode == 0) return qv != nullptr;
    if (mode == 1) return qsel && actions;
    if (mode == 2) return qsel && q_on != nullptr;
    return false;
  };
  if (!check_mode(qmode_on, qv_on, q_on)) return T2O_EINVAL;
  if ((qmode_on != 0 || (pack_tg && qmode_tg != 0)) && (n_actions < 1 || n_actions > MIX_MAXNA))
    return T2O_EUNSUPPORTED;
  a.net[0] = MixerNet{pack_on, hw0_on, hid_on, hid_sb, hid_st, q_on, qv_on, qmode_on, T_on,
                      y_on, hw_on, qvo_on, xout_on, xmid_on};
  int nnet = 1;
  if (pack_tg) {
    if (!hid_tg || !y_tg || !hw_tg || T_tg < 1 || !check_mode(qmode_tg, qv_tg, q_tg)) return T2O_EINVAL;
    a.net[1] = MixerNet{pack_tg, hw0_tg, hid_tg, hid_sb, hid_st, q_tg, qv_tg, qmode_tg, T_tg,
                        y_tg, hw_tg, qvo_tg, xout_tg, xmid_tg};
    nnet = 2;
  }
  // multi-tile mixers at a small batch: the recurrence decoupled (t2o_mixer_split.hip)
  a.t0 = phase == 1 ? t0 : 0;
  a.t1 = phase == 1 ? t1 : 0;
  if (const int r = t2o::mixer_split_fwd(a, nnet, (hipStream_t)stream, phase); r != 1) return r;
  if (phase) return T2O_EUNSUPPORTED;
  int rc = T2O_EUNSUPPORTED;
  T2O_DISPATCH_MIXER(L->E, L->H, L->D, L->n_ent, L->FF, L->pos_func == T2O_POS_ABS,
                     rc = (L->prec ? launch_mixer_fwd<E_, H_, D_, NE_, FF_, RTM_, __bf16>(a, nnet, (hipStream_t)stream)
                                   : launch_mixer_fwd<E_, H_, D_, NE_, FF_, RTM_, float>(a, nnet, (hipStream_t)stream)));
  return rc;
}

extern "C" int t2o_mixer_unroll_fwd(const t2o_mixer_fwd_args* a, void* stream) {
  if (!a || a->phase < 0 || a->phase > 2 || (a->phase == 1 && (a->t0 < 0 || a->t0 >= a->t1))) return T2O_EINVAL;
  const int ph = a->phase;
  return mixer_fwd_impl(a->L, a->pack_on, a->pack_tg, a->states, a->st_sb, a->st_st, a->hid_on, a->hid_tg, a->hid_sb,
                        a->hid_st, a->hw0_on, a->hw0_tg, a->qmode_on, a->qmode_tg, a->qv_on, a->qv_tg, a->q_on,
                        a->q_tg, a->q_ts, a->n_actions, a->actions, a->act_sb, a->act_st, a->avail, a->av_sb,
                        a->av_st, a->y_on, a->hw_on, a->qvo_on, a->xout_on, a->xmid_on, a->y_tg, a->hw_tg, a->qvo_tg,
                        a->xout_tg, a->xmid_tg, a->B, a->T_on, a->T_tg, ph, ph ? a->t0 : 0, ph ? a->t1 : 0, stream);
}

// worst case: 1 episode per workgroup, plus the decoupled multi-tile mixer's
// parallel workgroups (t2o_mixer_split.hip) at the batches it runs at
extern "C" int t2o_mixer_bwd_max_slabs(int B) { return B + t2o::mixer_split_extra_slabs(B); }

extern "C" int64_t t2o_mixer_bwd_work_floats(const t2o_layout* L, int B, int T) {
  if (!L || L->kind != 1 || B < 1 || T < 1) return -1;
  return t2o::mixer_split_work_floats(*L, B, T);
}

extern "C" int t2o_mixer_split(const t2o_layout* L, int B) {
  if (!L || L->kind != 1 || B < 1) return T2O_EINVAL;
  return t2o::mixer_split_taken(*L, B) ? 1 : 0;
}

static int mixer_bwd_impl(const t2o_layout* L, const float* pack, const float* states,
                                          int64_t st_sb, int64_t st_st, const float* hid, int64_t hid_sb,
                                          int64_t hid_st, const float* hw0, const float* qv, const float* hw,
                                          const float* xout, const float* xmid, const float* gy,
                                          const float* ghw_ext, float* gqv, float* ghid, float* ghw0,
                                          float* gslabs, int max_slabs, int* nslab, void* tape, float* work,
                                          int64_t work_floats, float* ghw_carry, int phase, int t_lo, int t_hi,
                                          int B, int T, void* stream) {
  if (phase < 0 || phase > 2) return T2O_EINVAL;
  if (!L || L->kind != 1 || !pack || !states || !hid || !qv || !hw || !xout || !gy || !gqv || !ghid ||
      !gslabs || !nslab || !tape || B < 1 || T < 1 || L->E > 64)
    return T2O_EINVAL;
  if (L->generic) {  // (no decoupled form: phases and ranges are the split kernels')
    if (phase) return T2O_EUNSUPPORTED;
    return gen_mixer_unroll_bwd(L, pack, states, st_sb, st_st, hid, hid_sb, hid_st, hw0, qv, hw, xout, xmid, gy,
                                ghw_ext, gqv, ghid, ghw0, gslabs, max_slabs, nslab, tape, B, T, (hipStream_t)stream);
  }
  MixerBwdArgs a{};
  a.f.L = *L;
  a.f.states = states;
  a.f.st_sb = st_sb;
  a.f.st_st = st_st;
  a.f.B = B;
  a.f.Fs = L->F;
  a.f.na = L->n_ent;
  a.f.net[0] = MixerNet{pack, hw0, hid, hid_sb, hid_st, nullptr, qv, 0, T, nullptr, nullptr, nullptr, nullptr,
                        nullptr};
  a.xmid = xmid;
  grad_layout(*L, a.G);
  a.hw = hw;
  a.xout = xout;
  a.gy = gy;
  a.ghw_ext = ghw_ext;
  a.gqv = gqv;
  a.ghid = ghid;
  a.ghw0 = ghw0;
  a.slabs = gslabs;
  a.tape = tape;
  if (const int r = t2o::mixer_split_bwd(a, work, work_floats, max_slabs, nslab, (hipStream_t)stream, phase, t_lo,
                                         phase == 2 ? t_hi : 0, ghw_carry);
      r != 1)
    return r;
  if (phase) return T2O_EUNSUPPORTED;
  int rc = T2O_EUNSUPPORTED;
  T2O_DISPATCH_MIXER(L->E, L->H, L->D, L->n_ent, L->FF, L->pos_func == T2O_POS_ABS,
                     rc = (L->prec ? launch_mixer_bwd<E_, H_, D_, NE_, FF_, RTM_, __bf16>(a, max_slabs, nslab, (hipStream_t)stream)
                                   : launch_mixer_bwd<E_, H_, D_, NE_, FF_, RTM_, float>(a, max_slabs, nslab, (hipStream_t)stream)));
  return rc;
}

extern "C" int t2o_mixer_unroll_bwd(const t2o_mixer_bwd_args* a, void* stream) {
  if (!a) return T2O_EINVAL;
  return mixer_bwd_impl(a->L, a->pack, a->states, a->st_sb, a->st_st, a->hid, a->hid_sb, a->hid_st, a->hw0, a->qv,
                        a->hw, a->xout, a->xmid, a->gy, a->ghw_ext, a->gqv, a->ghid, a->ghw0, a->gslabs, a->max_slabs,
                        a->nslab, a->tape, a->work, a->work_floats, a->ghw_carry, a->phase, a->t_lo, a->t_hi, a->B,
                        a->T, stream);
}
