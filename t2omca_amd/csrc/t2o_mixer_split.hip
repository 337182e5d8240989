// t2o_mixer_split.hip — the multi-tile mixers (A + 3 > 16 query rows: 14+
// AGVs) with their recurrence decoupled from the rest.
//
// Reference: n_transf_mixer.py:55-91.  Of the A + 3 query rows a mixer step
// reads out, only the 3 hyper tokens are recurrent (n_transf_mixer.py:69,91:
// they are the next step's hyper_weights).  The A agent rows (w1) attend over
// step t's keys — which hold the previous hyper tokens — but nothing of step
// t + 1 depends on them.  t2o_mixer.hip's one-wave kernels carry all ⌈(A+3)/16⌉
// query tiles through the recurrence; here:
//   forward   mixs_fwd_rec_kernel   per episode, t = 0..T-1: only the WINDOW,
//                                   the last 16 query rows [A+3-16, A+3) (the 3
//                                   hyper rows and the agents before them):
//                                   hw, the window's xout / xmid rows
//             mixs_fwd_rows_kernel  per (episode, step) of each network, all
//                                   independent: keys from the stored hw_{t-1},
//                                   the query rows before the window, then the
//                                   mixing head on all rows -> y, qv
//   backward  mixs_bwd_rows_kernel  per (episode, step), independent: the head's
//                                   backward (dL/dqvals, hyper_b2 grads, and the
//                                   window rows' grads without the carried hyper
//                                   part), the block backward of the rows before
//                                   the window (their tape records; their key
//                                   grads -> ghid, and the hyper keys' share)
//             mixs_bwd_rec_kernel   per episode, t = T-1..0: the window's block
//                                   backward with the carried hyper grads; adds
//                                   its key grads into ghid and carries the
//                                   hyper keys' total to step t - 1
// The recurrent kernels run ONE 16-row tile per step where t2o_mixer.hip's run
// all of them (two at 16 AGVs, five at 64): at a small replay batch, where a
// step's latency is the kernel's time, that halves (or better) the recurrence,
// and the parallel kernels fill the chip with b·T items.  Records (the compact
// per-block stream, (step, episode, query row) order), slabs and outputs mean
// what they mean in t2o_mixer.hip; the key-gradient sums run in another order.
#define T2O_SWZ_HOIST 0
#include <algorithm>
#include <cstdlib>

#include "t2o_dispatch.hpp"
#include "t2o_layout.hpp"
#include "t2o_mixer_block.hpp"
#include "t2o_mixer_parts.hpp"

using namespace t2o;

namespace {

// window rows [q0, q0 + 16) = the last 16 query rows; rows [0, q0) run in the
// parallel kernels as ⌈q0 / 16⌉ tiles (the last one partial)
T2O_DEV int mixs_q0(int nq) { return nq - 16; }

// the keys' inputs of step t only (state features, agent hidden tokens): what
// mix_keys reads of MixIn (the recurrent kernels need no Q selection)
template <int E, int A>
T2O_DEV void mixs_load_keys(const MixerFwdArgs& a, const MixerNet& n, int b, int t, MixIn<E, A>& in, int na) {
  using Dm = MixDims<E, A>;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  const float* st = a.states + b * a.st_sb + t * a.st_st;
#pragma unroll
  for (int s = 0; s < Dm::ST; ++s) {
    const int j = min(16 * s + c, na - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) in.st[s][r] = st[j * a.Fs + min(4 * g + r, a.Fs - 1)];
  }
  const float* hd = n.hid + b * n.hid_sb + t * n.hid_st;
#pragma unroll
  for (int k = 0; k < MixIn<E, A>::HV; ++k) in.hid[k] = ld4(hd + 4 * min(lane + 64 * k, na * E / 4 - 1));
}

template <int E>
constexpr int mixs_hw() { return (3 * E + 63) / 64; }

// ---------------------------------------------------------------------------
// forward, recurrent part: one wave per (episode, network)
template <int E, int A>
struct MixsFwdDims {
  using Dm = MixDims<E, A>;
  static constexpr int PERW = Dm::X0F + 16 * Dm::LDO;  // key block + the window's final rows
};

// LB: as mixer_fwd_kernel's (t2o_mixer.hip)
template <int E, int H, int D, int A, int FF, int RT, bool WLDS, typename WT, int LB = 512>
__global__ __launch_bounds__(LB) void mixs_fwd_rec_kernel(MixerFwdArgs args) {
  using Dm = MixDims<E, A>;
  constexpr int ET = E / 16, HW = mixs_hw<E>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const int w = wave_id();
  const MixerNet n = args.net[blockIdx.y];
  const t2o_layout L = kernel_layout<E, H, D, FF, WT>(args.L);
  const int na = RT == 1 ? args.na : A, nq = na + 3, lk = 2 * na + 3, q0 = mixs_q0(nq);
  const int lds_w = WLDS ? (int)((lds_weight_floats<WT>(L, L.fwd_total) + 15) / 16 * 16) : 0;
  Wts<WT> P0;
  if constexpr (WLDS) {
    P0 = stage_weights(smem, n.pack, L, L.fwd_total, WT{});
    __syncthreads();
  } else {
    P0 = global_weights(n.pack, L, WT{});
  }
  const int b = blockIdx.x * args.waves + w;
  // steps [ts, te) of this network (a range; the target network runs one step more)
  const int ts = args.t0, te = args.t1 > 0 ? min(args.t1, n.T) : n.T;
  if (b >= args.B || ts >= te) return;  // wave-uniform; no block barriers after this point
  float* X0 = smem + lds_w + w * MixsFwdDims<E, A>::PERW;
  float* OUT = X0 + Dm::X0F;  // window row c at OUT + c * LDO
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  for (int i = lane; i < Dm::X0F; i += 64) X0[i] = 0.f;
  // the hyper tokens entering step ts: hw0 / zeros, or what the range before wrote
  const float* hws = ts > 0 ? n.hw + ((size_t)b * n.T + ts - 1) * 3 * E : n.hw0 ? n.hw0 + (size_t)b * 3 * E : nullptr;
  for (int i = lane; i < 3 * E; i += 64) X0[(2 * na + i / E) * Dm::LDX + i % E] = hws ? hws[i] : 0.f;
  MixIn<E, A> in;
  mixs_load_keys<E, A>(args, n, b, ts, in, na);
  const int q = q0 + c;  // this lane's query row (always < nq)
  for (int t = ts; t < te; ++t) {
    const Wts<WT> P = step_view(P0);
    mix_keys<E, A>(P, L, in, X0, na);
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < te) mixs_load_keys<E, A>(args, n, b, t + 1, in, na);
    wave_sync();
    KeyFrags<E, Dm::KT, sizeof(WT) == 2> K;
    K.template load<Dm::LDX>(X0);
    f4 x[ET];
#pragma unroll
    for (int ft = 0; ft < ET; ++ft) x[ft] = ld4(X0 + (na + q) * Dm::LDX + 16 * ft + 4 * g);
    const size_t bt = (size_t)b * n.T + t;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (d > 0 && n.xmid) {
        float* xm = n.xmid + (((bt * (D - 1) + d - 1) * nq) + q) * E;
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) st4(xm + 16 * ft + 4 * g, x[ft]);
      }
      mixer_block_fwd<E, H, Dm::KT, FF, false>(P, L, d, K, lk, x, nullptr);
    }
    float* xo = n.xout + (bt * nq + q) * E;
#pragma unroll
    for (int ft = 0; ft < ET; ++ft) {
      st4(OUT + c * Dm::LDO + 16 * ft + 4 * g, x[ft]);
      st4(xo + 16 * ft + 4 * g, x[ft]);
    }
    wave_sync();
    // the hyper rows na..na+2 are window rows 13..15: outputs, and step t+1's keys
    float hv[HW];
#pragma unroll
    for (int k = 0; k < HW; ++k) {
      const int i = lane + 64 * k;
      hv[k] = i < 3 * E ? OUT[(13 + i / E) * Dm::LDO + i % E] : 0.f;
      if (i < 3 * E) n.hw[bt * 3 * E + i] = hv[k];
    }
    wave_sync();  // every X0 read of this step done (K, x) before the hyper rows change
#pragma unroll
    for (int k = 0; k < HW; ++k) {
      const int i = lane + 64 * k;
      if (i < 3 * E) X0[(2 * na + i / E) * Dm::LDX + i % E] = hv[k];
    }
    wave_sync();
  }
}

// ---------------------------------------------------------------------------
// forward, the rest: every (episode, step) of a network independently; a
// workgroup's waves loop over the network's items (the weights staged once)
template <int E, int A>
struct MixsRowsDims {
  using Dm = MixDims<E, A>;
  static constexpr int PERW = Dm::X0F + Dm::OUTF;  // key block + all final query rows
  static constexpr int XL = (16 * E + 63) / 64;    // the window's final rows, lane-indexed
};

template <int E, int A>
struct MixsRowsIn {
  MixIn<E, A> m;
  float hwp[mixs_hw<E>()];       // hw_{t-1} (hw0 / zeros at t = 0)
  float xl[MixsRowsDims<E, A>::XL];  // the window's final rows of step t (from the recurrent kernel)
};

template <int E, int A>
T2O_DEV void mixs_rows_load(const MixerFwdArgs& a, const MixerNet& n, int b, int t, MixsRowsIn<E, A>& in, int na) {
  const int lane = threadIdx.x & 63, nq = na + 3, q0 = mixs_q0(nq);
  mix_load<E, A>(a, n, b, t, in.m, na);
  const size_t bt = (size_t)b * n.T + t;
#pragma unroll
  for (int k = 0; k < mixs_hw<E>(); ++k) {
    const int i = min(lane + 64 * k, 3 * E - 1);
    in.hwp[k] = t > 0 ? n.hw[(bt - 1) * 3 * E + i] : (n.hw0 ? n.hw0[(size_t)b * 3 * E + i] : 0.f);
  }
#pragma unroll
  for (int k = 0; k < MixsRowsDims<E, A>::XL; ++k) in.xl[k] = n.xout[(bt * nq + q0) * E + lane + 64 * k];
}

template <int E, int H, int D, int A, int FF, int RT, bool WLDS, typename WT>
__global__ __launch_bounds__(512) void mixs_fwd_rows_kernel(MixerFwdArgs args) {
  using Dm = MixDims<E, A>;
  using Rd = MixsRowsDims<E, A>;
  constexpr int ET = E / 16, HW = mixs_hw<E>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const int w = wave_id();
  const MixerNet n = args.net[blockIdx.y];
  const t2o_layout L = kernel_layout<E, H, D, FF, WT>(args.L);
  const int na = RT == 1 ? args.na : A, nq = na + 3, lk = 2 * na + 3, q0 = mixs_q0(nq);
  const int pf = RT ? L.pos_func : T2O_POS_ABS;
  const float pb = RT ? L.pos_beta : 1.f;
  const int lds_w = WLDS ? (int)((lds_weight_floats<WT>(L, L.fwd_total) + 15) / 16 * 16) : 0;
  Wts<WT> P0;
  if constexpr (WLDS) {
    P0 = stage_weights(smem, n.pack, L, L.fwd_total, WT{});
    __syncthreads();
  } else {
    P0 = global_weights(n.pack, L, WT{});
  }
  const int items = args.B * n.T;
  const int stride = gridDim.x * args.waves;
  int it = blockIdx.x * args.waves + w;
  if (it >= items) return;  // wave-uniform; no block barriers after this point
  float* X0 = smem + lds_w + w * Rd::PERW;
  float* OUT = X0 + Dm::X0F;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  for (int i = lane; i < Dm::X0F; i += 64) X0[i] = 0.f;
  const int ntp = (q0 + 15) / 16;  // tiles before the window
  MixsRowsIn<E, A> in;
  mixs_rows_load<E, A>(args, n, it / n.T, it % n.T, in, na);
  for (; it < items; it += stride) {
    const int b = it / n.T, t = it % n.T;
    const size_t bt = (size_t)b * n.T + t;
    const Wts<WT> P = step_view(P0);
    mix_keys<E, A>(P, L, in.m, X0, na);
#pragma unroll
    for (int k = 0; k < HW; ++k) {
      const int i = lane + 64 * k;
      if (i < 3 * E) X0[(2 * na + i / E) * Dm::LDX + i % E] = in.hwp[k];
    }
#pragma unroll
    for (int k = 0; k < Rd::XL; ++k) {
      const int i = lane + 64 * k;
      OUT[(q0 + i / E) * Dm::LDO + i % E] = in.xl[k];
    }
    const float myq = mix_qv<E, A>(n, in.m, args.n_actions, args.avail != nullptr);
    __builtin_amdgcn_sched_barrier(0);  // this item's inputs consumed before the next item's are loaded
    if (it + stride < items) mixs_rows_load<E, A>(args, n, (it + stride) / n.T, (it + stride) % n.T, in, na);
    wave_sync();
    KeyFrags<E, Dm::KT, sizeof(WT) == 2> K;
    K.template load<Dm::LDX>(X0);
    for (int qt = 0; qt < ntp; ++qt) {
      const int q = 16 * qt + c;
      const bool qv_ = q < q0;
      f4 x[ET];
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) x[ft] = qv_ ? ld4(X0 + (na + q) * Dm::LDX + 16 * ft + 4 * g) : zero4();
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const Wts<WT> Pq = step_view(P);  // (opaque per query tile: weight reads stay in the loop)
        if (d > 0 && n.xmid && qv_) {
          float* xm = n.xmid + (((bt * (D - 1) + d - 1) * nq) + q) * E;
#pragma unroll
          for (int ft = 0; ft < ET; ++ft) st4(xm + 16 * ft + 4 * g, x[ft]);
        }
        mixer_block_fwd<E, H, Dm::KT, FF, false>(Pq, L, d, K, lk, x, nullptr);
      }
      if (qv_) {
        float* xo = n.xout + (bt * nq + q) * E;
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) {
          st4(OUT + q * Dm::LDO + 16 * ft + 4 * g, x[ft]);
          st4(xo + 16 * ft + 4 * g, x[ft]);
        }
      }
    }
    wave_sync();
    float qv[A];
    bcast_agents<A>(myq, qv);
    float pre_h, pre2;
    const float y = mixer_head<E, A>(P, L, OUT, qv, pre_h, pre2, na, pf, pb);
    if (lane == 0) n.y[bt] = y;
    if (n.qv && lane < na) n.qv[bt * na + lane] = myq;
    wave_sync();  // OUT / X0 read before the next item writes them
  }
}

// ---------------------------------------------------------------------------
// backward.  Workspace: goutl [B][T][16][E] (window rows' grads, non-recurrent
// part), pghw [B][T][3][E] (the hyper keys' grads from the rows before the
// window)
struct MixsBwdArgs {
  MixerBwdArgs m;
  float* goutl;
  float* pghw;
  int slab0;  // first slab of this kernel's workgroups
  // the recurrent kernel: steps t_hi - 1 .. t_lo; ghw_carry [B][3][E] hands the
  // hyper grads from one range to the next (ranges run from the last down); the
  // range starting at T - 1 clears its slabs and zeroes the tape's tail
  int t_lo, t_hi;
  float* ghw_carry;
};

template <int E, int H, int D, int A, int FF, int RT, bool WLDS, typename WT>
__global__ __launch_bounds__(256) void mixs_bwd_rows_kernel(MixsBwdArgs sa) {
  using Dm = MixDims<E, A>;
  constexpr int KM = key_mode<Dm::KT, WT>();
  using Bd = MixBwdDims<E, A, KM>;
  constexpr int ET = E / 16, KT = Dm::KT;
  static_assert(Dm::QT > 1, "multi-tile mixers only");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const MixerBwdArgs& args = sa.m;
  const MixerFwdArgs& fa = args.f;
  const MixerNet& n = fa.net[0];
  const t2o_layout& L = fa.L;
  const t2o_layout& G = args.G;
  const int na = RT == 1 ? fa.na : A, nq = na + 3, lk = 2 * na + 3, q0 = mixs_q0(nq);
  const int w = wave_id();
  float* X0 = smem + args.lds_w + w * Bd::PERW;
  float* X0T = X0 + Dm::X0F;        // (KM 1: the transposed key block)
  float* GOUT = X0T + Bd::X0TF;     // head grads, rows of OUT layout (stride LDB)
  float* stage = GOUT + Bd::GOUT;   // final rows (head) / staging / gX0 region
  float* gs = args.slabs + (size_t)(sa.slab0 + blockIdx.x) * G.grad_total;
  Wts<WT> P0 = WLDS ? stage_weights(smem, n.pack, L, L.fwd_total, WT{}) : global_weights(n.pack, L, WT{});
  P0.vol = false;
  zero_flushed_regions(gs, G, false);
  __syncthreads();
  const int T = n.T, items = fa.B * T, stride = gridDim.x * args.waves;
  const int it0 = blockIdx.x * args.waves + w;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  using Rec = TapeRec<E, H, FF>;
  const size_t nrec = (size_t)fa.B * T * nq, ctiles = (nrec + 15) / 16;
  const int f = lane < E ? lane : 0;
  const bool fv = lane < E;
  f4 gWe[ET];
#pragma unroll
  for (int ft = 0; ft < ET; ++ft) gWe[ft] = zero4();
  f4 ln2[D][2 * ET];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int t = 0; t < 2 * ET; ++t) ln2[d][t] = zero4();
  float gWo = 0.f, gbo = 0.f;
  const int ntp = (q0 + 15) / 16;
  if (it0 < items) {
    for (int i = lane; i < Dm::X0F; i += 64) X0[i] = 0.f;
    for (int it = it0; it < items; it += stride) {
      const int b = it / T, t = it % T;
      const size_t bt = (size_t)b * T + t;
      const Wts<WT> P = step_view(P0);
      MixBwdIn<E, A, D> cur;
      mixb_load<E, A, D, false>(args, n, b, t, cur, na);
      mix_keys<E, A>(P, L, cur.m, X0, na);
#pragma unroll
      for (int k = 0; k < MixBwdIn<E, A, D>::HW; ++k) {
        const int i = lane + 64 * k;
        if (i < 3 * E) X0[(2 * na + i / E) * Dm::LDX + i % E] = cur.hwp[k];
      }
      float* OUT = stage;
#pragma unroll
      for (int k = 0; k < MixBwdIn<E, A, D>::XO; ++k) {
        const int i = lane + 64 * k;
        if (i < nq * E) OUT[(i / E) * Bd::LDB + i % E] = cur.xo[k];
      }
      wave_sync();
      // ---- mixing head backward without the carried hyper grads
      const float ghw0[3] = {0.f, 0.f, 0.f};
      mixer_head_bwd<E, A, WT, Bd::LDB>(P, L, OUT, GOUT, cur.m.qs[0], cur.gy, ghw0, args.gqv + bt * na + lane, gWo,
                                        gbo, na, RT ? L.pos_func : T2O_POS_ABS, RT ? L.pos_beta : 1.f);
      for (int i = nq * Bd::LDB + lane; i < Bd::OUTB; i += 64) GOUT[i] = 0.f;
      wave_sync();
      // the window rows' grads for the recurrent kernel
      for (int i = lane; i < 16 * E; i += 64) sa.goutl[bt * 16 * E + i] = GOUT[(q0 + i / E) * Bd::LDB + i % E];
      KeyFrags<E, KT, sizeof(WT) == 2, KM> K;
      load_keys<Dm::LDX>(K, X0, X0T);
      f4 gX0[KT][ET];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) gX0[kt][ft] = zero4();
#pragma unroll 1
      for (int qt = 0; qt < ntp; ++qt) {
        const int q = 16 * qt + c;
        const bool qv_ = q < q0;
        f4 gx[ET];
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) gx[ft] = qv_ ? ld4(GOUT + q * Bd::LDB + 16 * ft + 4 * g) : zero4();
#pragma unroll
        for (int d = D - 1; d >= 0; --d) {
        const Wts<WT> Pq = step_view(P);  // (opaque per query tile: weight reads stay in the loop)
          f4 x[ET];
#pragma unroll
          for (int ft = 0; ft < ET; ++ft) x[ft] = qv_ ? ld4(X0 + (na + q) * Dm::LDX + 16 * ft + 4 * g) : zero4();
          if (d > 0) {
            if (args.xmid) {
#pragma unroll
              for (int ft = 0; ft < ET; ++ft)
                x[ft] = qv_ ? ld4(args.xmid + ((bt * (D - 1) + d - 1) * nq + q) * E + 16 * ft + 4 * g) : zero4();
            } else {
              for (int dd = 0; dd < d; ++dd) mixer_block_fwd<E, H, KT, FF, false>(Pq, L, dd, K, lk, x, nullptr);
            }
          }
          WT* tile = static_cast<WT*>(args.tape) + ((size_t)d * ctiles * 16 + ((size_t)t * fa.B + b) * nq + 16 * qt) * Rec::SIZE;
          MixerCacheLean<E, H, KT, FF> cache;
          const MaskedRec<WT, 2> rec(tile, min(16, q0 - 16 * qt), Rec::SIZE);
          mixer_block_fwd_lean<E, H, KT, FF>(Pq, L, d, K, lk, x, cache, rec);
          mixer_block_bwd_lean<E, H, KT, FF>(Pq, L, gs, rec, stage, d, K, lk, gX0, cache, gx, ln2[d]);
        }
        wave_sync();
#pragma unroll
        for (int ft = 0; ft < ET; ++ft)
          if (qv_) st4(GOUT + q * Bd::LDB + 16 * ft + 4 * g, gx[ft]);
      }
      // ---- state embedding grads from this item's key-grad share
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
      float* GX0 = stage;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft)
#pragma unroll
          for (int r = 0; r < 4; ++r) GX0[(16 * kt + 4 * g + r) * Bd::LDB + 16 * ft + c] = gX0[kt][ft][r];
      wave_sync();
      // the query path of the rows before the window (all agents: q < q0 <= na)
      for (int qt = 0; qt < ntp; ++qt) {
        const int q = 16 * qt + c;
        if (q < q0) {
#pragma unroll
          for (int ft = 0; ft < ET; ++ft) {
            float* dst = GX0 + (na + q) * Bd::LDB + 16 * ft + 4 * g;
            st4(dst, ld4(dst) + ld4(GOUT + q * Bd::LDB + 16 * ft + 4 * g));
          }
        }
      }
      wave_sync();
      for (int i = lane; i < na * E / 4; i += 64)
        st4(args.ghid + bt * na * E + 4 * i, ld4(GX0 + (na + 4 * i / E) * Bd::LDB + (4 * i) % E));
      for (int i = lane; i < 3 * E; i += 64) sa.pghw[bt * 3 * E + i] = GX0[(2 * na + i / E) * Bd::LDB + i % E];
      wave_sync();
    }
  }
  flush_in_wave_order([&] {
    if (it0 < items) {
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

// the window's per-step inputs, prefetched a step ahead
template <int E, int A>
struct MixsRecIn {
  static constexpr int GL = (16 * E + 63) / 64;
  MixIn<E, A> m;
  float hwp[mixs_hw<E>()];
  float gl[GL];     // goutl of step t: window rows' grads, lane-indexed
  float ph[3];      // pghw of step t, lane = feature
  float ghx[3];     // ghw_ext of step t, lane = feature
  f4 stT[MixDims<E, A>::ST];
  f4 gh[MixIn<E, A>::HV];  // ghid of step t as the parallel kernel left it, f4 i = lane + 64k of [A][E]
};

template <int E, int A>
T2O_DEV void mixs_rec_load(const MixsBwdArgs& sa, const MixerNet& n, int b, int t, MixsRecIn<E, A>& in, int na) {
  using Dm = MixDims<E, A>;
  const MixerBwdArgs& args = sa.m;
  const MixerFwdArgs& fa = args.f;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  mixs_load_keys<E, A>(fa, n, b, t, in.m, na);
  const size_t bt = (size_t)b * n.T + t;
#pragma unroll
  for (int k = 0; k < mixs_hw<E>(); ++k) {
    const int i = min(lane + 64 * k, 3 * E - 1);
    in.hwp[k] = t > 0 ? args.hw[(bt - 1) * 3 * E + i] : (n.hw0 ? n.hw0[(size_t)b * 3 * E + i] : 0.f);
  }
#pragma unroll
  for (int k = 0; k < MixsRecIn<E, A>::GL; ++k) in.gl[k] = sa.goutl[bt * 16 * E + lane + 64 * k];
  const int fl = lane < E ? lane : 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    in.ph[k] = sa.pghw[(bt * 3 + k) * E + fl];
    in.ghx[k] = args.ghw_ext ? args.ghw_ext[(bt * 3 + k) * E + fl] : 0.f;
  }
  const float* st = fa.states + b * fa.st_sb + t * fa.st_st;
#pragma unroll
  for (int s = 0; s < Dm::ST; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * s + 4 * g + r;
      float v = ld_or0(st, j * fa.Fs + c, j < na && c < fa.Fs);
      if (j < na && c == fa.Fs) v = 1.f;
      in.stT[s][r] = v;
    }
  // (a step ahead: read-modify-written at the step's end, a dependent load there
  // would expose its latency on the recurrence)
#pragma unroll
  for (int k = 0; k < MixIn<E, A>::HV; ++k) in.gh[k] = ld4(args.ghid + bt * na * E + 4 * min(lane + 64 * k, na * E / 4 - 1));
}

template <int E, int H, int D, int A, int FF, int RT, bool WLDS, typename WT>
__global__ __launch_bounds__(256) void mixs_bwd_rec_kernel(MixsBwdArgs sa) {
  using Dm = MixDims<E, A>;
  constexpr int KM = key_mode<Dm::KT, WT>();
  using Bd = MixBwdDims<E, A, KM>;
  constexpr int ET = E / 16, KT = Dm::KT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const MixerBwdArgs& args = sa.m;
  const MixerFwdArgs& fa = args.f;
  const MixerNet& n = fa.net[0];
  const t2o_layout& L = fa.L;
  const t2o_layout& G = args.G;
  const int na = RT == 1 ? fa.na : A, nq = na + 3, lk = 2 * na + 3, q0 = mixs_q0(nq);
  const int w = wave_id();
  float* X0 = smem + args.lds_w + w * Bd::PERW;
  float* X0T = X0 + Dm::X0F;   // (KM 1: the transposed key block)
  float* GW = X0T + Bd::X0TF;  // the window rows' grads [16][LDB] (ghw staging first)
  float* stage = GW + Bd::GOUT;
  float* gs = args.slabs + (size_t)(sa.slab0 + blockIdx.x) * G.grad_total;
  Wts<WT> P0 = WLDS ? stage_weights(smem, n.pack, L, L.fwd_total, WT{}) : global_weights(n.pack, L, WT{});
  P0.vol = false;
  const int T = n.T;
  const int t_lo = sa.t_lo, t_hi = sa.t_hi > 0 ? sa.t_hi : T;
  if (t_hi == T) zero_flushed_regions(gs, G, false);
  __syncthreads();
  const int b = blockIdx.x * args.waves + w;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  using Rec = TapeRec<E, H, FF>;
  const size_t nrec = (size_t)fa.B * T * nq, ctiles = (nrec + 15) / 16;
  if (blockIdx.x == 0 && w == 0 && t_hi == T) {  // zero each block's compact stream past its last record
    const int tail = (int)(ctiles * 16 - nrec) * Rec::SIZE;
    for (int d = 0; d < D; ++d) {
      WT* z = static_cast<WT*>(args.tape) + ((size_t)d * ctiles * 16 + nrec) * Rec::SIZE;
      for (int i = lane; i < tail; i += 64) z[i] = WT(0.f);
    }
  }
  const int f = lane < E ? lane : 0;
  const bool fv = lane < E;
  f4 gWe[ET];
#pragma unroll
  for (int ft = 0; ft < ET; ++ft) gWe[ft] = zero4();
  f4 ln2[D][2 * ET];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int t = 0; t < 2 * ET; ++t) ln2[d][t] = zero4();
  if (b < fa.B) {
    for (int i = lane; i < Dm::X0F; i += 64) X0[i] = 0.f;
    float ghw[3] = {0.f, 0.f, 0.f};  // grad wrt this step's hyper outputs, lane = feature
    if (t_hi < T) {  // from the range after this one
#pragma unroll
      for (int k = 0; k < 3; ++k) ghw[k] = fv ? sa.ghw_carry[((size_t)b * 3 + k) * E + f] : 0.f;
    }
    const int q = q0 + c;            // this lane's window row
    MixsRecIn<E, A> cur;
    mixs_rec_load<E, A>(sa, n, b, t_hi - 1, cur, na);
    for (int t = t_hi - 1; t >= t_lo; --t) {
      const Wts<WT> P = step_view(P0);
      const size_t bt = (size_t)b * T + t;
      mix_keys<E, A>(P, L, cur.m, X0, na);
#pragma unroll
      for (int k = 0; k < mixs_hw<E>(); ++k) {
        const int i = lane + 64 * k;
        if (i < 3 * E) X0[(2 * na + i / E) * Dm::LDX + i % E] = cur.hwp[k];
      }
      // window rows' grads: the parallel kernel's part, plus the carried hyper
      // grads on rows 13..15 (the hyper rows na..na+2)
#pragma unroll
      for (int k = 0; k < 3; ++k) ghw[k] += cur.ghx[k];
#pragma unroll
      for (int k = 0; k < MixsRecIn<E, A>::GL; ++k) {
        const int i = lane + 64 * k;
        GW[(i / E) * Bd::LDB + i % E] = cur.gl[k];
      }
      wave_sync();
      if (fv) {
#pragma unroll
        for (int h = 0; h < 3; ++h) GW[(13 + h) * Bd::LDB + f] += ghw[h];
      }
      const MixsRecIn<E, A> now = cur;  // (the prefetch below overwrites cur)
      __builtin_amdgcn_sched_barrier(0);
      if (t > t_lo) mixs_rec_load<E, A>(sa, n, b, t - 1, cur, na);
      wave_sync();
      KeyFrags<E, KT, sizeof(WT) == 2, KM> K;
      load_keys<Dm::LDX>(K, X0, X0T);
      f4 gX0[KT][ET];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) gX0[kt][ft] = zero4();
      f4 gx[ET];
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) gx[ft] = ld4(GW + c * Bd::LDB + 16 * ft + 4 * g);
#pragma unroll
      for (int d = D - 1; d >= 0; --d) {
        f4 x[ET];
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) x[ft] = ld4(X0 + (na + q) * Dm::LDX + 16 * ft + 4 * g);
        if (d > 0) {
          if (args.xmid) {
#pragma unroll
            for (int ft = 0; ft < ET; ++ft) x[ft] = ld4(args.xmid + ((bt * (D - 1) + d - 1) * nq + q) * E + 16 * ft + 4 * g);
          } else {
            for (int dd = 0; dd < d; ++dd) mixer_block_fwd<E, H, KT, FF, false>(P, L, dd, K, lk, x, nullptr);
          }
        }
        WT* tile = static_cast<WT*>(args.tape) + ((size_t)d * ctiles * 16 + ((size_t)t * fa.B + b) * nq + q0) * Rec::SIZE;
        MixerCacheLean<E, H, KT, FF> cache;
        const MaskedRec<WT, 2> rec(tile, 16, Rec::SIZE);
        mixer_block_fwd_lean<E, H, KT, FF>(P, L, d, K, lk, x, cache, rec);
        mixer_block_bwd_lean<E, H, KT, FF>(P, L, gs, rec, stage, d, K, lk, gX0, cache, gx, ln2[d]);
      }
      // ---- state embedding grads
#pragma unroll
      for (int s = 0; s < Dm::ST; ++s)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) {
          f4 am;
#pragma unroll
          for (int r = 0; r < 4; ++r) am[r] = 16 * s + 4 * g + r < na ? gX0[s][ft][r] : 0.f;
          if constexpr (sizeof(WT) == 2) {
            gWe[ft] = mfma_b16(to_bf4(am), to_bf4(now.stT[s]), gWe[ft]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) gWe[ft] = mfma4(am[r], now.stT[s][r], gWe[ft]);
          }
        }
      wave_sync();
      float* GX0 = stage;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft)
#pragma unroll
          for (int r = 0; r < 4; ++r) GX0[(16 * kt + 4 * g + r) * Bd::LDB + 16 * ft + c] = gX0[kt][ft][r];
      wave_sync();
      // the window rows' query path
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) {
        float* dst = GX0 + (na + q) * Bd::LDB + 16 * ft + 4 * g;
        st4(dst, ld4(dst) + gx[ft]);
      }
      wave_sync();
      // agent hidden tokens: the parallel kernel's share + this one's
#pragma unroll
      for (int k = 0; k < MixIn<E, A>::HV; ++k) {
        const int i = lane + 64 * k;
        if (i < na * E / 4)
          st4(args.ghid + bt * na * E + 4 * i, now.gh[k] + ld4(GX0 + (na + 4 * i / E) * Bd::LDB + (4 * i) % E));
      }
      // the hyper keys' total: the grad wrt the hyper outputs of step t - 1
#pragma unroll
      for (int k = 0; k < 3; ++k) ghw[k] = fv ? GX0[(2 * na + k) * Bd::LDB + f] + now.ph[k] : 0.f;
      wave_sync();
    }
    float* const gout = t_lo > 0 ? sa.ghw_carry : args.ghw0;
    if (gout && fv) {
#pragma unroll
      for (int k = 0; k < 3; ++k) gout[((size_t)b * 3 + k) * E + f] = ghw[k];
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
      ln2_flush<E, D>(gs, G, ln2);
    }
  });
}

// ---------------------------------------------------------------------------
// The window's BPTT on two waves per episode, one per transformer block (depth
// 2), as t2o_mixer.hip's mixer_bwd_pipe_kernel does for the one-tile mixers:
//   block-1 wave: keys+fwd1(t) | bwd1(t) | keys+fwd1(t-1) | bwd1(t-1) | ...
//   block-0 wave:      -       | fwd0(t) |     bwd0(t)    | fwd0(t-1) | ...
// so the recomputes come off the dependent chain bwd1 -> bwd0 -> (hyper grads)
// -> bwd1 ...  Per step the block-1 wave starts from the window rows' grads (the
// parallel kernel's share + the carried hyper grads: no head here), the block-0
// wave finishes with the step's key grads (its own + the parallel kernel's hyper
// share) and the ghid read-modify-write.  One pair per workgroup: the two waves
// land on two SIMDs and each may take the whole register file (the small batches
// this runs at leave SIMDs idle anyway).  Pair LDS: the key block X0 (written by
// the block-1 recompute, read by both recomputes) and a region R owned by the
// wave in its backward phase: the window grads / dW staging, then the hand-over
// 1 -> 0 (block-1 key grads in rows < lk, the grads wrt the block-1 input past
// them), then the step's total key grads, whose hyper rows the block-1 wave reads
// at its next backward phase.
template <int E, int A>
struct MixsPipeDims {
  using Dm = MixDims<E, A>;
  using Bd = MixBwdDims<E, A>;
  static constexpr int LDR = E;
  static constexpr int XCH = Dm::LKCAP * LDR;  // window-row grads after the key rows
  static constexpr int R0 = Bd::STAGE > Dm::KT * 16 * LDR ? Bd::STAGE : Dm::KT * 16 * LDR;
  static constexpr int REGION = R0 > XCH + 16 * LDR ? R0 : XCH + 16 * LDR;
  static constexpr int PAIRF = Dm::X0F + REGION;
};

template <int E, int A>
T2O_DEV void mixs_load_stT(const MixerFwdArgs& fa, int b, int t, f4 (&stT)[MixDims<E, A>::ST], int na) {
  const int c = lane_c(), g = lane_g();
  const float* st = fa.states + b * fa.st_sb + t * fa.st_st;
#pragma unroll
  for (int s = 0; s < MixDims<E, A>::ST; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * s + 4 * g + r;
      float v = ld_or0(st, j * fa.Fs + c, j < na && c < fa.Fs);
      if (j < na && c == fa.Fs) v = 1.f;
      stT[s][r] = v;
    }
}

template <int E, int H, int A, int FF, typename WT>
T2O_DEV void mixs_pipe_block1(const MixsBwdArgs& sa, const Wts<WT>& P0, const t2o_layout& L, const t2o_layout& G,
                              float* __restrict__ gs, float* X0, float* R, int b, PairBarrier& pbar, int na) {
  const MixerBwdArgs& args = sa.m;
  const t2o_layout Lb = block_view(L, 1), Gb = block_view(G, 1);
  using Dm = MixDims<E, A>;
  using Pd = MixsPipeDims<E, A>;
  using Rec = TapeRec<E, H, FF>;
  constexpr int ET = E / 16, KT = Dm::KT, HW = mixs_hw<E>(), GL = (16 * E + 63) / 64;
  constexpr bool BF = sizeof(WT) == 2;
  const MixerFwdArgs& fa = args.f;
  const MixerNet& n = fa.net[0];
  const int T = n.T, t_lo = sa.t_lo, t_hi = sa.t_hi;
  const int nq = na + 3, lk = 2 * na + 3, q0 = mixs_q0(nq);
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  const int f = lane < E ? lane : 0;
  const bool fv = lane < E;
  const size_t ctiles = ((size_t)fa.B * T * nq + 15) / 16;
  f4 ln2[2 * ET];
#pragma unroll
  for (int i = 0; i < 2 * ET; ++i) ln2[i] = zero4();
  for (int t = t_hi - 1; t >= t_lo; --t) {
    const size_t bt = (size_t)b * T + t;
    const MaskedRec<WT> rec(static_cast<WT*>(args.tape) + (1 * ctiles * 16 + ((size_t)t * fa.B + b) * nq + q0) * Rec::SIZE,
                            16, Rec::SIZE);
    MixerCacheLean<E, H, KT, FF> cache;
    KeyFrags<E, KT, BF> K;
    MixIn<E, A> in;
    float hwp[HW], gl[GL], ghx[3];
    f4 xm[ET];
    {  // ---- recompute: the key block of step t, block-1 forward of the window rows
      mixs_load_keys<E, A>(fa, n, b, t, in, na);
#pragma unroll
      for (int k = 0; k < HW; ++k) {
        const int i = min(lane + 64 * k, 3 * E - 1);
        hwp[k] = t > 0 ? args.hw[(bt - 1) * 3 * E + i] : (n.hw0 ? n.hw0[(size_t)b * 3 * E + i] : 0.f);
      }
#pragma unroll
      for (int k = 0; k < GL; ++k) gl[k] = sa.goutl[bt * 16 * E + lane + 64 * k];
#pragma unroll
      for (int k = 0; k < 3; ++k) ghx[k] = args.ghw_ext ? args.ghw_ext[(bt * 3 + k) * E + f] : 0.f;
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) xm[ft] = ld4(args.xmid + (bt * nq + q0 + c) * E + 16 * ft + 4 * g);
      const Wts<WT> P = step_view(P0);
      mix_keys<E, A>(P, L, in, X0, na);
#pragma unroll
      for (int k = 0; k < HW; ++k) {
        const int i = lane + 64 * k;
        if (i < 3 * E) X0[(2 * na + i / E) * Dm::LDX + i % E] = hwp[k];
      }
      wave_sync();
      K.template load<Dm::LDX>(X0);
      f4 x[ET];
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) x[ft] = xm[ft];
      mixer_block_fwd_lean<E, H, KT, FF>(P, Lb, 0, K, lk, x, cache, rec);
    }
    pbar.sync();
    {  // ---- backward: the window rows' grads, block 1
      const Wts<WT> P = step_view(P0);
      float ghw[3];  // grad wrt this step's hyper outputs: the step after's key grads (block-0 wave), carried
#pragma unroll
      for (int k = 0; k < 3; ++k)
        ghw[k] = !fv ? 0.f : t < t_hi - 1 ? R[(2 * na + k) * Pd::LDR + f]
                           : t_hi < T ? sa.ghw_carry[((size_t)b * 3 + k) * E + f] : 0.f;
      wave_sync();
#pragma unroll
      for (int k = 0; k < GL; ++k) {
        const int i = lane + 64 * k;
        R[(i / E) * Pd::LDR + i % E] = gl[k];
      }
      wave_sync();
      if (fv) {
#pragma unroll
        for (int k = 0; k < 3; ++k) R[(13 + k) * Pd::LDR + f] += ghw[k] + ghx[k];
      }
      wave_sync();
      f4 gx[ET];
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) gx[ft] = ld4(R + c * Pd::LDR + 16 * ft + 4 * g);
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
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) st4(R + Pd::XCH + c * Pd::LDR + 16 * ft + 4 * g, gx[ft]);
    }
    pbar.sync();
  }
  pbar.sync();  // the block-0 wave's last backward phase
  flush_in_wave_order([&] {
    vec_accumulate_g<ET>(gs + Gb.g2[0], &ln2[0]);
    vec_accumulate_g<ET>(gs + Gb.n2[0], &ln2[ET]);
  });
  (void)G;
}

template <int E, int H, int A, int FF, typename WT>
T2O_DEV void mixs_pipe_block0(const MixsBwdArgs& sa, const Wts<WT>& P0, const t2o_layout& L, const t2o_layout& G,
                              float* __restrict__ gs, const float* X0, float* R, int b, PairBarrier& pb, int na) {
  const MixerBwdArgs& args = sa.m;
  const t2o_layout Lb = block_view(L, 0), Gb = block_view(G, 0);
  using Dm = MixDims<E, A>;
  using Pd = MixsPipeDims<E, A>;
  using Rec = TapeRec<E, H, FF>;
  constexpr int ET = E / 16, KT = Dm::KT, HV = MixIn<E, A>::HV;
  constexpr bool BF = sizeof(WT) == 2;
  const MixerFwdArgs& fa = args.f;
  const int T = fa.net[0].T, t_lo = sa.t_lo, t_hi = sa.t_hi;
  const int nq = na + 3, lk = 2 * na + 3, q0 = mixs_q0(nq);
  const size_t ctiles = ((size_t)fa.B * T * nq + 15) / 16;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  const int f = lane < E ? lane : 0;
  const bool fv = lane < E;
  f4 ln2[2 * ET], gWe[ET];
#pragma unroll
  for (int i = 0; i < ET; ++i) ln2[i] = ln2[ET + i] = gWe[i] = zero4();
  pb.sync();  // one phase behind the block-1 wave
  for (int t = t_hi - 1; t >= t_lo; --t) {
    const size_t bt = (size_t)b * T + t;
    const MaskedRec<WT> rec(static_cast<WT*>(args.tape) + (((size_t)t * fa.B + b) * nq + q0) * Rec::SIZE, 16,
                            Rec::SIZE);
    MixerCacheLean<E, H, KT, FF> cache;
    KeyFrags<E, KT, BF> K;
    f4 stT[Dm::ST], gh[HV];
    float ph[3];
    {  // ---- recompute: block-0 forward of the window rows (block inputs = X0 rows na + q)
      mixs_load_stT<E, A>(fa, b, t, stT, na);
#pragma unroll
      for (int k = 0; k < HV; ++k) gh[k] = ld4(args.ghid + bt * na * E + 4 * min(lane + 64 * k, na * E / 4 - 1));
#pragma unroll
      for (int k = 0; k < 3; ++k) ph[k] = sa.pghw[(bt * 3 + k) * E + f];
      const Wts<WT> P = step_view(P0);
      K.template load<Dm::LDX>(X0);
      f4 x[ET];
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) x[ft] = ld4(X0 + (na + q0 + c) * Dm::LDX + 16 * ft + 4 * g);
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
      for (int ft = 0; ft < ET; ++ft) gx[ft] = ld4(R + Pd::XCH + c * Pd::LDR + 16 * ft + 4 * g);
      wave_sync();
      mixer_block_bwd_lean<E, H, KT, FF>(P, Lb, gs, rec, R, 0, K, lk, gX0, cache, gx, ln2);
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
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) {  // the window rows' query path
        float* dst = R + (na + q0 + c) * Pd::LDR + 16 * ft + 4 * g;
        st4(dst, ld4(dst) + gx[ft]);
      }
      wave_sync();
#pragma unroll
      for (int k = 0; k < HV; ++k) {  // agent hidden tokens: the parallel kernel's share + the window's
        const int i = lane + 64 * k;
        if (i < na * E / 4)
          st4(args.ghid + bt * na * E + 4 * i, gh[k] + ld4(R + (na + 4 * i / E) * Pd::LDR + (4 * i) % E));
      }
      // the hyper keys' total (+ the parallel kernel's share): the block-1 wave's
      // carried grads at t - 1, or what this range hands on
      if (fv) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float v = R[(2 * na + k) * Pd::LDR + f] + ph[k];
          R[(2 * na + k) * Pd::LDR + f] = v;
          if (t == t_lo) {
            float* gout = t_lo > 0 ? sa.ghw_carry : args.ghw0;
            if (gout) gout[((size_t)b * 3 + k) * E + f] = v;
          }
        }
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
  (void)G;
}

template <int E, int H, int D, int A, int FF, int RT, typename WT>
__global__ __launch_bounds__(128) void mixs_bwd_rec_pipe_kernel(MixsBwdArgs sa) {
  static_assert(D == 2, "one wave per block of a depth-2 stack");
  using Dm = MixDims<E, A>;
  using Pd = MixsPipeDims<E, A>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  T2O_LDS_POISON(smem);
  const MixerBwdArgs& args = sa.m;
  const t2o_layout& L = args.f.L;
  const t2o_layout& G = args.G;
  const int na = RT == 1 ? args.f.na : A;
  const int w = __builtin_amdgcn_readfirstlane(wave_id());  // 0: block 1, 1: block 0
  float* X0 = smem + args.lds_w;
  float* R = X0 + Dm::X0F;
  float* gs = args.slabs + (size_t)(sa.slab0 + blockIdx.x) * G.grad_total;
  const int T = args.f.net[0].T;
  const Wts<WT> P0 = stage_weights(smem, args.f.net[0].pack, L, sizeof(WT) == 4 ? L.fwd_total : L.total, WT{}, false);
  if (sa.t_hi == T) zero_flushed_regions(gs, G, false);
  for (int i = threadIdx.x; i < Dm::X0F; i += 128) X0[i] = 0.f;
  int* const flags = reinterpret_cast<int*>(R + Pd::REGION);
  if (threadIdx.x < PAIR_FLAG_FLOATS) flags[threadIdx.x] = 0;
  if (blockIdx.x == 0 && threadIdx.x < 64 && sa.t_hi == T) {  // zero each block's compact stream past its last record
    using Rec = TapeRec<E, H, FF>;
    const size_t nrec = (size_t)args.f.B * T * (na + 3), ctiles = (nrec + 15) / 16;
    const int tail = (int)(ctiles * 16 - nrec) * Rec::SIZE;
    for (int dd = 0; dd < D; ++dd) {
      WT* z = static_cast<WT*>(args.tape) + ((size_t)dd * ctiles * 16 + nrec) * Rec::SIZE;
      for (int i = threadIdx.x; i < tail; i += 64) z[i] = WT(0.f);
    }
  }
  __syncthreads();
  PairBarrier pb = PairBarrier::make(flags, w);
  const int b = blockIdx.x;
  if (w == 0) {
    __builtin_amdgcn_s_setprio(1);  // (the head of the dependent chain, as the one-tile pipeline's block-1 wave)
    mixs_pipe_block1<E, H, A, FF, WT>(sa, P0, L, G, gs, X0, R, b, pb, na);
  } else {
    mixs_pipe_block0<E, H, A, FF, WT>(sa, P0, L, G, gs, X0, R, b, pb, na);
  }
}

// T2O_MIXS_REC=single: the one-wave recurrent backward (A/B, cross-check)
inline bool mixs_rec_single() {
  const char* e = getenv("T2O_MIXS_REC");
  return e && e[0] == 's';
}

// ---------------------------------------------------------------------------
// launchers

// When the split runs: multi-tile instances, a replay batch small enough that
// the one-wave kernels leave most SIMDs idle.  T2O_MIXER_SPLIT=0 / 1 forces it
// off / on (A/B timing, cross-checks).
constexpr int MIXS_AUTO_MAX_EPISODES = 256;
inline int mixs_env() {  // (read per call: tests switch it within one process)
  const char* e = getenv("T2O_MIXER_SPLIT");
  return e ? (e[0] == '1' ? 1 : e[0] == '0' ? 0 : -1) : -1;
}
inline bool mixs_wanted(int B) {
  const int e = mixs_env();
  return e >= 0 ? e == 1 : B <= MIXS_AUTO_MAX_EPISODES;
}
constexpr int MIXS_ROWS_MAX_WG = 512;  // workgroups of the parallel backward (= its slabs)

inline int resident_grid(const void* kern, int threads, size_t lds, int want) {
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) == hipSuccess &&
      hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      per_cu > 0 && cus > 0)
    return std::max(1, std::min(want, per_cu * cus));
  return want;
}

template <int E, int H, int D, int A, int FF, int RT, typename WT>
int mixs_launch_fwd(const MixerFwdArgs& args, int nnet, hipStream_t stream, int phase) {
  using Dm = MixDims<E, A>;
  if (!kernel_layout_matches<E, H, D, FF, WT>(args.L)) return T2O_EINVAL;
  const size_t wfl = (lds_weight_floats<WT>(args.L, args.L.fwd_total) + 15) / 16 * 16;
  // recurrent part
  if (phase != 2) {
    MixerFwdArgs a = args;
    constexpr size_t perw = MixsFwdDims<E, A>::PERW;
    size_t lds = 0;
    for (a.waves = 8, a.wlds = 1; a.waves >= 2; a.waves >>= 1) {
      lds = sizeof(float) * (wfl + a.waves * perw);
      if (lds <= 160 * 1024) break;
    }
    if (a.waves < 2) {
      a.waves = 4;
      a.wlds = 0;
      lds = sizeof(float) * 4 * perw;
    }
    // (small batches: fewer waves per workgroup spread the episodes over more CUs)
    while (a.waves > 1 && (args.B + a.waves - 1) / a.waves * nnet < 256) a.waves >>= 1;
    if (a.wlds) lds = sizeof(float) * (wfl + a.waves * perw);
    else lds = sizeof(float) * a.waves * perw;
    const bool wide = a.waves <= 4 && 2 * lds > 160 * 1024;  // one workgroup per CU: one wave per SIMD
    auto kern = wide ? (a.wlds ? mixs_fwd_rec_kernel<E, H, D, A, FF, RT, true, WT, 256>
                               : mixs_fwd_rec_kernel<E, H, D, A, FF, RT, false, WT, 256>)
                     : (a.wlds ? mixs_fwd_rec_kernel<E, H, D, A, FF, RT, true, WT>
                               : mixs_fwd_rec_kernel<E, H, D, A, FF, RT, false, WT>);
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3((args.B + a.waves - 1) / a.waves, nnet), dim3(64 * a.waves), lds, stream, a);
    const int rc = (int)hipGetLastError();
    if (rc) return rc;
  }
  // every (episode, step)
  if (phase == 1) return 0;
  {
    MixerFwdArgs a = args;
    constexpr size_t perw = MixsRowsDims<E, A>::PERW;
    size_t lds = 0;
    for (a.waves = 8, a.wlds = 1; a.waves >= 2; a.waves >>= 1) {
      lds = sizeof(float) * (wfl + a.waves * perw);
      if (lds <= 160 * 1024) break;
    }
    if (a.waves < 2) {
      a.waves = 4;
      a.wlds = 0;
      lds = sizeof(float) * 4 * perw;
      if (lds > 160 * 1024) return T2O_EUNSUPPORTED;
    }
    auto kern = a.wlds ? mixs_fwd_rows_kernel<E, H, D, A, FF, RT, true, WT> : mixs_fwd_rows_kernel<E, H, D, A, FF, RT, false, WT>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    int tmax = args.net[0].T;
    if (nnet > 1) tmax = std::max(tmax, args.net[1].T);
    const int want = (args.B * tmax + a.waves - 1) / a.waves;  // workgroups per network
    const int grid = std::max(1, std::min(want, resident_grid((const void*)kern, 64 * a.waves, lds, 1 << 20) / nnet));
    hipLaunchKernelGGL(kern, dim3(grid, nnet), dim3(64 * a.waves), lds, stream, a);
    return (int)hipGetLastError();
  }
}

template <int E, int H, int D, int A, int FF, int RT, typename WT>
int mixs_launch_bwd(MixsBwdArgs& sa, int max_slabs, int* nslab, hipStream_t stream, int phase) {
  using Bd = MixBwdDims<E, A, key_mode<MixDims<E, A>::KT, WT>()>;  // (the rows / one-wave kernels' buffers)
  MixerBwdArgs& args = sa.m;
  if (!kernel_layout_matches<E, H, D, FF, WT>(args.f.L)) return T2O_EINVAL;
  const t2o_layout& L = args.f.L;
  const int lds_w = (int)((lds_weight_floats<WT>(L, L.fwd_total) + 15) / 16 * 16);
  auto pick = [&](int maxw, int& waves, bool& wlds, size_t& lds) {
    const MixLaunch m = mix_pick((size_t)lds_w, Bd::PERW, maxw, 1, maxw, 1);
    waves = m.waves;
    wlds = m.wlds;
    lds = m.lds;
    return m.waves >= 1;
  };
  const int B = args.f.B, T = args.f.net[0].T;
  // parallel part first: ghid partial, the window grads, the hyper keys' share
  int g2 = 0;
  {
    int waves;
    bool wlds;
    size_t lds;
    if (!pick(4, waves, wlds, lds)) return T2O_EUNSUPPORTED;
    args.waves = waves;
    args.lds_w = wlds ? lds_w : 0;
    auto kern = wlds ? mixs_bwd_rows_kernel<E, H, D, A, FF, RT, true, WT> : mixs_bwd_rows_kernel<E, H, D, A, FF, RT, false, WT>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int want = (B * T + waves - 1) / waves;
    g2 = std::min(resident_grid((const void*)kern, 64 * waves, lds, want), MIXS_ROWS_MAX_WG);
    sa.slab0 = 0;
    if (g2 > max_slabs) return T2O_EINVAL;
    if (phase != 2) {
      hipLaunchKernelGGL(kern, dim3(g2), dim3(64 * waves), lds, stream, sa);
      const int rc = (int)hipGetLastError();
      if (rc) return rc;
    }
  }
  // the recurrence over the window: two waves per episode (one per block) where the
  // block inputs are stored and the weights fit LDS beside the pair's buffers
  if constexpr (D == 2) {
    const int lds_wp = (int)((lds_weight_floats<WT>(L, sizeof(WT) == 4 ? L.fwd_total : L.total) + 15) / 16 * 16);
    const size_t lds = sizeof(float) * ((size_t)lds_wp + MixsPipeDims<E, A>::PAIRF + PAIR_FLAG_FLOATS);
    if (args.xmid && lds <= 160 * 1024 && !mixs_rec_single()) {
      args.lds_w = lds_wp;
      sa.slab0 = g2;
      if (g2 + B > max_slabs) return T2O_EINVAL;
      *nslab = g2 + B;
      if (phase == 1) return 0;
      auto kern = mixs_bwd_rec_pipe_kernel<E, H, D, A, FF, RT, WT>;
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(kern, dim3(B), dim3(128), lds, stream, sa);
      return (int)hipGetLastError();
    }
  }
  {
    int waves;
    bool wlds;
    size_t lds;
    if (!pick(4, waves, wlds, lds)) return T2O_EUNSUPPORTED;
    while (waves > 1 && (B + waves - 1) / waves < 256) waves >>= 1;  // spread small batches over CUs
    lds = sizeof(float) * ((wlds ? (size_t)lds_w : 0) + waves * Bd::PERW);
    args.waves = waves;
    args.lds_w = wlds ? lds_w : 0;
    const int g1 = (B + waves - 1) / waves;
    sa.slab0 = g2;
    if (g2 + g1 > max_slabs) return T2O_EINVAL;
    *nslab = g2 + g1;
    if (phase == 1) return 0;
    auto kern = wlds ? mixs_bwd_rec_kernel<E, H, D, A, FF, RT, true, WT> : mixs_bwd_rec_kernel<E, H, D, A, FF, RT, false, WT>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(g1), dim3(64 * waves), lds, stream, sa);
    return (int)hipGetLastError();
  }
}

template <int E, int H, int D, int NE, int FF, int RTM>
int mixs_fwd_dispatch(const MixerFwdArgs& a, int nnet, hipStream_t stream, int phase) {
  if constexpr (MixDims<E, NE>::QT > 1)
    return a.L.prec ? mixs_launch_fwd<E, H, D, NE, FF, RTM, __bf16>(a, nnet, stream, phase)
                    : mixs_launch_fwd<E, H, D, NE, FF, RTM, float>(a, nnet, stream, phase);
  return 1;
}
template <int E, int H, int D, int NE, int FF, int RTM>
int mixs_bwd_dispatch(MixsBwdArgs& sa, int max_slabs, int* nslab, hipStream_t stream, int phase) {
  if constexpr (MixDims<E, NE>::QT > 1)
    return sa.m.f.L.prec ? mixs_launch_bwd<E, H, D, NE, FF, RTM, __bf16>(sa, max_slabs, nslab, stream, phase)
                         : mixs_launch_bwd<E, H, D, NE, FF, RTM, float>(sa, max_slabs, nslab, stream, phase);
  return 1;
}

}  // namespace

namespace t2o {

// t2o_mixer.hip's entry points call these for the multi-tile instances; 1 = not
// taken (the one-wave kernels run)
int mixer_split_fwd(const MixerFwdArgs& a, int nnet, hipStream_t stream, int phase) {
  if (!mixs_wanted(a.B) || !a.net[0].xout || (nnet > 1 && !a.net[1].xout)) return 1;
  int rc = 1;
  T2O_DISPATCH_MIXER(a.L.E, a.L.H, a.L.D, a.L.n_ent, a.L.FF, a.L.pos_func == T2O_POS_ABS,
                     rc = (mixs_fwd_dispatch<E_, H_, D_, NE_, FF_, RTM_>(a, nnet, stream, phase)));
  return rc;
}

int64_t mixer_split_work_floats(const t2o_layout& L, int B, int T) {
  if (L.generic || L.n_ent + 3 <= 16) return 0;
  return (int64_t)B * T * 19 * L.E;  // goutl [B][T][16][E] + pghw [B][T][3][E]
}

int mixer_split_bwd(const MixerBwdArgs& m, float* work, int64_t work_floats, int max_slabs, int* nslab,
                    hipStream_t stream, int phase, int t_lo, int t_hi, float* ghw_carry) {
  const int B = m.f.B, T = m.f.net[0].T;
  const int64_t need = mixer_split_work_floats(m.f.L, B, T);
  if (!mixs_wanted(B) || !work || need <= 0 || work_floats < need) return 1;
  if (t_hi <= 0) t_hi = T;
  if (t_lo < 0 || t_lo >= t_hi || t_hi > T || ((t_lo > 0 || t_hi < T) && !ghw_carry)) return T2O_EINVAL;
  MixsBwdArgs sa{};
  sa.m = m;
  sa.goutl = work;
  sa.pghw = work + (int64_t)B * T * 16 * m.f.L.E;
  sa.t_lo = t_lo;
  sa.t_hi = t_hi;
  sa.ghw_carry = ghw_carry;
  int rc = 1;
  T2O_DISPATCH_MIXER(m.f.L.E, m.f.L.H, m.f.L.D, m.f.L.n_ent, m.f.L.FF, m.f.L.pos_func == T2O_POS_ABS,
                     rc = (mixs_bwd_dispatch<E_, H_, D_, NE_, FF_, RTM_>(sa, max_slabs, nslab, stream, phase)));
  return rc;
}

bool mixer_split_taken(const t2o_layout& L, int B) {
  return !L.generic && L.n_ent + 3 > 16 && mixs_wanted(B);
}

int mixer_split_extra_slabs(int B) { return mixs_wanted(B) ? MIXS_ROWS_MAX_WG : 0; }

}  // namespace t2o
