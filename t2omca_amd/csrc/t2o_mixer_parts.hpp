// t2o_mixer_parts.hpp — what the mixer kernels share (t2o_mixer.hip: one wave
// per episode; t2o_mixer_split.hip: the multi-tile mixers decoupled into the
// hyper-token recurrence and the per-(episode, step) agent rows): argument
// blocks, compile-time dims, the per-step input loads, the key block, and the
// mixing head forward / backward.  Reference: n_transf_mixer.py:55-103.
#pragma once
#include <algorithm>
#include <cstdlib>

#include "t2o_layout.hpp"
#include "t2o_mixer_block.hpp"

namespace t2o {


struct MixerNet {
  const float* pack;
  const float* hw0;   // [B][3][E] or null (zeros)
  const float* hid;   // [b][t][a][E] (a-stride E)
  int64_t hid_sb, hid_st;
  const float* qsel;  // Q values for qmode 1/2: [b][t][a][NA], time extent q_ts
  const float* qv_in; // qmode 0: [B][T][A]
  int qmode, T;
  float* y;           // [B][T]
  float* hw;          // [B][T][3][E]
  float* qv;          // [B][T][A] (may be null)
  float* xout;        // [B][T][A+3][E] final query outputs (may be null)
  float* xmid;        // [B][T][D-1][A+3][E] inputs of blocks 1..D-1 (may be null)
};

struct MixerFwdArgs {
  t2o_layout L;
  MixerNet net[2];
  const float* states;  // [b][t][ns*Fs]
  int64_t st_sb, st_st;
  const float* qarg;    // online-agent Q for the double-Q argmax, [b][t][a][NA]
  int q_ts, n_actions;
  const int64_t* actions;
  int64_t act_sb, act_st;
  const int32_t* avail;  // [b][t][a][NA]
  int64_t av_sb, av_st;
  int B, Fs;
  int na;           // agents = state entities (n_entities = n_agents)
  int waves, wlds;  // set by the launcher
  int t0, t1;       // decoupled recurrence only (t2o_mixer_split.hip): steps [t0, t1); t1 = 0: all
};

// Compile-time dims of an instance for A agents — the exact count, or the
// capacity of a runtime-agent instance (t2o_dispatch.hpp), which sizes its
// register arrays and LDS buffers for A and runs na <= A agents: the kernel
// code indexes with the runtime counts
//   na (state entities = agents), nq = na + 3 (query rows read out: A weight
//   rows + 3 hyper tokens), lk = 2 na + 3 (keys; padding keys score -inf),
// X0 rows [0, na) state entities, [na, 2na) agent hidden tokens, [2na, 2na+3)
// hyper tokens; query row q is X0 row na + q.
template <int E, int A>
struct MixDims {
  static constexpr int QCAP = A + 3;        // query rows
  static constexpr int LKCAP = 2 * A + 3;   // keys
  static constexpr int KT = (LKCAP + 15) / 16;
  static constexpr int QT = (QCAP + 15) / 16;
  static constexpr int ST = (A + 15) / 16;
  static constexpr int LDX = E + 4;
  // row stride of the [row][feature] LDS blocks (final query rows, their grads, the
  // key grads): E + 4 floats, so the T-layout accesses (lane c = row, 16-B chunk
  // 4g of features) spread the 16 rows over distinct banks — at stride E = 32 a
  // ds_write_b128 of 8 rows hit one 4-bank set (8-way) and a ds_read_b128 4-way
  static constexpr int LDO = E + 4;
  static constexpr int X0F = KT * 16 * LDX;
  static constexpr int OUTF = QT * 16 * LDO;
  static constexpr int GX0F = KT * 16 * LDO;
  // forward: with one query tile the final query rows are complete only after
  // every key read of the step, so they can live in the key block itself
  static constexpr int FWD_PERW = X0F + (QT == 1 ? 0 : OUTF);
};

// Σ over lanes 0..E-1 (lane = feature; other lanes must hold 0), wave-uniform:
// DPP row sums put each 16-lane row's total in its lane 15, then scalar reads.
template <int E>
T2O_DEV float feat_sum(float v) {
  v = rowsum16_fast(v);
  float s = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 15));
#pragma unroll
  for (int r = 1; r < (E + 15) / 16; ++r) s += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16 * r + 15));
  return s;
}

// ELU (alpha 1): x > 0 ? x : e^x - 1.  e^x - 1 is v_exp_f32's e^x minus 1, or for
// |x| < 1/16, where that difference would cancel, its Taylor series to x^5 (next
// term < 2e-9 relative); libm's expm1f was ~20 VALU per lane per step.  Absolute
// error < 2e-7, far inside the fp32 parity bar.
T2O_DEV float elu1(float x) {
  if (x > 0.f) return x;
  const float small = x * (1.f + x * (0.5f + x * (1.f / 6.f + x * (1.f / 24.f + x * (1.f / 120.f)))));
  return x > -0.0625f ? small : exp_fast(x) - 1.f;
}

constexpr int MIX_MAXNA = 8;  // n_actions bound of the register-resident Q rows (launcher checks)

// Inputs of one (episode, step) that do not depend on the recurrence, loaded
// a step AHEAD into registers so their HBM latency hides behind the current
// step's compute:
//   st   state features in the embedding's T-layout (row j = 16s + c,
//        features 4g + r)
//   hid  the agents' hidden tokens, f4 i = lane + 64k of the [A][E] block
//   qs / qa / act   (lane a < A only) what the learner's Q selection needs:
//        qmode 0 qs[0] = qvals; 1 qs = Q row, act = action;
//        2 qs = target Q row, qa = online Q row masked by avail
template <int E, int A>
struct MixIn {
  using Dm = MixDims<E, A>;
  static constexpr int HV = (A * E / 4 + 63) / 64;
  f4 st[Dm::ST];
  f4 hid[HV];
  float qs[MIX_MAXNA], qa[MIX_MAXNA];
  int av[MIX_MAXNA];
  int act;
};

template <int E, int A>
T2O_DEV void mix_load(const MixerFwdArgs& a, const MixerNet& n, int b, int t, MixIn<E, A>& in, int na) {
  using Dm = MixDims<E, A>;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  // Every load is unconditional (in-bounds duplicates for padding lanes / rows /
  // action slots) and its register is left alone until the step that uses it:
  // a select right after a load would wait for it — and, the vector-memory
  // counter being in order, for every store issued before it — defeating the
  // prefetch.  Padding is harmless where it lands: state features past Fs meet
  // the zero-padded embedding columns, rows past NS / hidden lanes past A·E/4
  // are never stored (mix_keys), action slots past NA are masked in mix_qv.
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
  // per-agent inputs, lane a < A holds agent a's.  No branch on the Q-selection
  // mode either (a branch makes the loop-carried registers phis, and the
  // compiler then copies them — waiting for the loads — right after issuing):
  // fields a mode does not use load an in-bounds dummy.
  const int la = lane < na ? lane : na - 1;
  const int NA = a.n_actions > 0 ? a.n_actions : 1;
  const bool q0 = n.qmode == 0;
  const size_t qrow = q0 ? ((size_t)b * n.T + t) * na + la : (((size_t)b * a.q_ts + t) * na + la) * NA;
  const float* qsrc = q0 ? n.qv_in : n.qsel;
#pragma unroll
  for (int k = 0; k < MIX_MAXNA; ++k) in.qs[k] = qsrc[qrow + (q0 ? 0 : (k < NA ? k : NA - 1))];
  const bool q2 = n.qmode == 2, q1 = n.qmode == 1;
  const float* qa = q2 ? a.qarg + qrow : qsrc + qrow;
#pragma unroll
  for (int k = 0; k < MIX_MAXNA; ++k) in.qa[k] = qa[q2 ? (k < NA ? k : NA - 1) : 0];
  const int32_t* av = (q2 && a.avail) ? a.avail + b * a.av_sb + t * a.av_st + la * NA
                                      : reinterpret_cast<const int32_t*>(qsrc + qrow);
#pragma unroll
  for (int k = 0; k < MIX_MAXNA; ++k) in.av[k] = av[(q2 && a.avail) ? (k < NA ? k : NA - 1) : 0];
  const int32_t* ap = q1 ? reinterpret_cast<const int32_t*>(a.actions + b * a.act_sb + t * a.act_st + la)
                         : reinterpret_cast<const int32_t*>(qsrc + qrow);
  in.act = *ap;  // (low word of the int64 action)
}

// This lane's agent's mixer input (lane a < A): chosen-action Q (qmode 1) or
// the target Q at the avail-masked online argmax (qmode 2, first max wins).
template <int E, int A>
T2O_DEV float mix_qv(const MixerNet& n, const MixIn<E, A>& in, int NA, bool avail) {
  if (n.qmode == 0) return in.qs[0];
  int act = 0;
  if (n.qmode == 1) {
    act = in.act;
  } else {
    float qa[MIX_MAXNA];
#pragma unroll
    for (int k = 0; k < MIX_MAXNA; ++k)
      qa[k] = k < NA ? (avail && in.av[k] == 0 ? -9999999.0f : in.qa[k]) : -INFINITY;
    float best = qa[0];
#pragma unroll
    for (int k = 1; k < MIX_MAXNA; ++k)
      if (qa[k] > best) {
        best = qa[k];
        act = k;
      }
  }
  // a select chain, kept opaque per step: folded into qs[act] it would turn the
  // whole prefetch struct into a dynamically indexed scratch array
  float v = in.qs[0];
#pragma unroll
  for (int k = 1; k < MIX_MAXNA; ++k) {
    v = act == k ? in.qs[k] : v;
    asm volatile("" : "+v"(v));
  }
  return v;
}

// every lane gets all A agents' values (lane a holds agent a's): scalar broadcast
template <int A>
T2O_DEV void bcast_agents(float mine, float (&qv)[A]) {
#pragma unroll
  for (int ag = 0; ag < A; ++ag) qv[ag] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine), ag));
}

// Key block X0 rows for one step from the prefetched inputs: state-entity
// embeddings and agent hidden tokens (the hyper-token rows are carried in X0).
template <int E, int A, typename WT, typename In, bool HOIST = T2O_SWZ_HOIST>
T2O_DEV void mix_keys(const Wts<WT>& P, const t2o_layout& L, const In& in, float* X0, int na) {
  using Dm = MixDims<E, A>;
  constexpr int ET = E / 16;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < Dm::ST; ++s) {
    const int j = 16 * s + c;
    f4 emb[ET];
    matvec<ET, 1, HOIST>(P.w + L.We, 16, &in.st[s], emb, P.vol);
    if (j < na) {
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) st4(X0 + j * Dm::LDX + 16 * ft + 4 * g, emb[ft] + vec_t(P.v + L.be, ft));
    }
  }
#pragma unroll
  for (int k = 0; k < MixIn<E, A>::HV; ++k) {
    const int i = lane + 64 * k;
    if (i < na * E / 4) st4(X0 + (na + (4 * i) / E) * Dm::LDX + (4 * i) % E, in.hid[k]);
  }
}

// Mixing head (n_transf_mixer.py:75-89, pos_func abs: t2o_layout_init lays out
// every other qmix_pos_func generic) on the final query rows OUT[q][f],
// lanes = features.  Returns y; writes hyper tokens back into X0.
// (qv: capacity-sized; entries ag >= na are not read; LDO: OUT's row stride;
// pf / pb: qmix_pos_func and its softplus beta, n_transf_mixer.py:95-103 — the
// exact instances pass the constant abs, the runtime-entity ones the layout's)
template <int E, int A, typename WT, int LDO = MixDims<E, A>::LDO>
T2O_DEV float mixer_head(const Wts<WT>& P, const t2o_layout& L, const float* OUT,
                         const float (&qv)[A], float& pre_h, float& pre2, int na, int pf, float pb) {
  const int f = threadIdx.x & 63;
  const bool fv = f < E;
  const int fc = fv ? f : 0;
  float ph = OUT[na * LDO + fc];
#pragma unroll
  for (int ag = 0; ag < A; ++ag)
    if (ag < na) ph += qv[ag] * posf(OUT[ag * LDO + fc], pf, pb);
  pre_h = ph;
  const float hidden = elu1(ph);
  const float w2 = posf(OUT[(na + 1) * LDO + fc], pf, pb);
  const float yv = feat_sum<E>(fv ? hidden * w2 : 0.f);
  const float p2 = feat_sum<E>(fv ? P.s(L.Wo + fc) * OUT[(na + 2) * LDO + fc] : 0.f) + P.v[L.bo];
  pre2 = p2;
  return yv + fmaxf(p2, 0.f);
}


struct MixerBwdArgs {
  MixerFwdArgs f;     // net[0] = the network (qmode 0: qv_in = forward qv output)
  t2o_layout G;
  const float* hw;    // forward hw output [B][T][3][E]
  const float* xout;  // forward final query rows [B][T][A+3][E]
  const float* gy;    // [B][T]
  const float* ghw_ext;  // [B][T][3][E] extra grad on the hyper outputs (may be null)
  float* gqv;         // [B][T][A]
  float* ghid;        // [B][T][A][E]
  float* ghw0;        // [B][3][E] (may be null)
  const float* xmid;  // forward block inputs of blocks 1..D-1 [B][T][D-1][A+3][E] (may be null)
  float* slabs;
  void* tape;         // [D][T][B][QT][TapeRec::SIZE][16] in the MFMA operand type
  int lds_w;          // floats of LDS taken by the weights
  int waves;          // episodes (waves) per workgroup: 4, 2 or 1, whatever fits in LDS
};


// The backward's per-step inputs (all forward outputs or replay data, none
// recurrent), prefetched one step ahead like MixIn.
template <int E, int A, int D>
struct MixBwdIn {
  using Dm = MixDims<E, A>;
  static constexpr int ET = E / 16;
  static constexpr int HW = (3 * E + 63) / 64;
  static constexpr int XO = (Dm::QCAP * E + 63) / 64;
  MixIn<E, A> m;
  float hwp[HW];  // X0 hyper rows: hyper outputs of step t-1 (hw0 / zeros at t = 0)
  float xo[XO];   // forward final query rows of step t
  float ghx[3];   // ghw_ext of step t, lane = feature
  float gy;       // dL/dy of step t
  f4 xm[Dm::QT][D > 1 ? D - 1 : 1][ET];  // stored inputs of blocks 1..D-1 (T-layout query rows)
  f4 stT[Dm::ST];  // lane (g, c) reg r: state feature c of entity 16s + 4g + r; column Fs = 1 (bias)
};

template <int E, int A, int D, bool XM = true>
T2O_DEV void mixb_load(const MixerBwdArgs& args, const MixerNet& n, int b, int t, MixBwdIn<E, A, D>& in, int na) {
  using Dm = MixDims<E, A>;
  using In = MixBwdIn<E, A, D>;
  const MixerFwdArgs& fa = args.f;
  const int c = lane_c(), g = lane_g(), lane = threadIdx.x & 63;
  const int nq = na + 3;
  mix_load<E, A>(fa, n, b, t, in.m, na);
  const size_t bt = (size_t)b * n.T + t;
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
  if (XM && D > 1 && args.xmid) {
#pragma unroll
    for (int qt = 0; qt < Dm::QT; ++qt) {
      const int q = 16 * qt + c;
#pragma unroll
      for (int d = 1; d < D; ++d)
#pragma unroll
        for (int ft = 0; ft < In::ET; ++ft)
          in.xm[qt][d - 1][ft] =
              q < nq ? ld4(args.xmid + ((bt * (D - 1) + d - 1) * nq + q) * E + 16 * ft + 4 * g) : zero4();
    }
  }
  const float* st = fa.states + b * fa.st_sb + t * fa.st_st;
#pragma unroll
  for (int s = 0; s < Dm::ST; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * s + 4 * g + r;
      float v = 0.f;
      v = ld_or0(st, j * fa.Fs + c, j < na && c < fa.Fs);
      if (j < na && c == fa.Fs) v = 1.f;
      in.stT[s][r] = v;
    }
}

template <int E, int A, int KM = 0>
struct MixBwdDims {
  using Dm = MixDims<E, A>;
  // KM 1: the transposed key block X0T of LDS-read key fragments (KeyFrags) after X0
  static constexpr int X0TF = KM ? E * (16 * Dm::KT + 4) : 0;
  static constexpr int ET = E / 16, KT = Dm::KT;
  static constexpr int NSTAGE = (KT < ET ? KT : ET) < 2 ? 2 : (KT < ET ? KT : ET);
  static constexpr int STAGE = StageDims<NSTAGE>::FLOATS;
  // WORK holds, in turn: the final query rows (head forward), their grads, the
  // dW staging area (blocks), and the key-token grad block gX0 [KT*16][E].
  // With one query tile the grads are in registers before staging starts, so
  // the three uses can alias; otherwise the grads keep their own region.
  // row stride of the [row][feature] blocks: padded (Dm::LDO) with one query tile;
  // the multi-tile kernels keep stride E — padded, the 64-AGV kernel's per-wave
  // buffers no longer fit two waves per workgroup beside the weights
  static constexpr int LDB = Dm::QT == 1 ? Dm::LDO : E;
  static constexpr int OUTB = Dm::QT * 16 * LDB;
  static constexpr int GX0B = KT * 16 * LDB;
  static constexpr int GOUT = Dm::QT == 1 ? 0 : OUTB;
  static constexpr int W0 = OUTB > STAGE ? OUTB : STAGE;
  static constexpr int WORK = GOUT + (W0 > GX0B ? W0 : GX0B);
  static constexpr int PERW = Dm::X0F + X0TF + WORK;
};

// Mixing-head backward of one (episode, step), lanes = features
// (n_transf_mixer.py:75-89, pos_func abs): from the final query rows OUT (rows
// [0, nq), stride E) and dL/dy, writes the grads wrt those rows to GOUT (may
// alias OUT), lane a < na's dL/dqvals[a] to gqv, and accumulates the hyper_b2
// grads.  ghw: grads wrt the step's hyper outputs (carried + external).
template <int E, int A, typename WT, int LDO = MixDims<E, A>::LDO>
T2O_DEV void mixer_head_bwd(const Wts<WT>& P, const t2o_layout& L, const float* OUT, float* GOUT, float myq,
                            float gyv, const float (&ghw)[3], float* gqv, float& gWo, float& gbo, int na, int pf,
                            float pb) {
  const int lane = threadIdx.x & 63;
  const int f = lane < E ? lane : 0;
  const bool fv = lane < E;
  float qv[A];
  bcast_agents<A>(myq, qv);
  float pre_h, pre2;
  (void)mixer_head<E, A, WT, LDO>(P, L, OUT, qv, pre_h, pre2, na, pf, pb);
  const float hidden = elu1(pre_h);
  const float xw2 = OUT[(na + 1) * LDO + f];
  float pw2, sgn_w2;
  posd(xw2, pf, pb, pw2, sgn_w2);
  const float gpre = gyv * pw2 * (pre_h > 0.f ? 1.f : hidden + 1.f);  // ELU': e^x = (e^x - 1) + 1
  const float gpre2 = pre2 > 0.f ? gyv : 0.f;
  // gout[0, A): the agents' weight rows (entries >= na unused); gout[A + k]: hyper row na + k
  float gout[A + 3];
  float gqm = 0.f;  // lane a < na: dL/dqvals[a]
#pragma unroll
  for (int ag = 0; ag < A; ++ag) {
    if (ag < na) {
      const float xa = OUT[ag * LDO + f];
      float pa, da;
      posd(xa, pf, pb, pa, da);
      gout[ag] = qv[ag] * gpre * da;
      const float gq = feat_sum<E>(fv ? gpre * pa : 0.f);
      gqm = lane == ag ? gq : gqm;
    }
  }
  if (lane < na) *gqv = gqm;
  gout[A] = gpre + ghw[0];
  gout[A + 1] = gyv * hidden * sgn_w2 + ghw[1];
  const float x2 = OUT[(na + 2) * LDO + f];
  gout[A + 2] = gpre2 * P.s(L.Wo + f) + ghw[2];
  gWo += gpre2 * x2;
  gbo += gpre2;
  wave_sync();  // every OUT read done (GOUT may alias it)
  if (fv) {
#pragma unroll
    for (int q = 0; q < A + 3; ++q) {
      if (q < na) GOUT[q * LDO + f] = gout[q];
      else if (q >= A) GOUT[(q - A + na) * LDO + f] = gout[q];
    }
  }
}

}  // namespace t2o

namespace t2o {
// t2o_mixer_split.hip: the multi-tile mixers' recurrence decoupled from the rest
// (small replay batches).  The entry points return 1 when the split does not
// apply (t2o_mixer.hip's one-wave kernels run instead), else a status.
// phase (both): 0 the whole unroll; forward 1 the recurrence over steps
// [a.t0, a.t1) only, 2 the parallel rows only (after every range of the
// recurrence); backward 1 the parallel rows only, 2 the recurrence over steps
// t_hi - 1 .. t_lo only (ranges from the last down; ghw_carry [B][3][E] carries
// the hyper grads between them)
int mixer_split_fwd(const MixerFwdArgs& a, int nnet, hipStream_t stream, int phase = 0);
int mixer_split_bwd(const MixerBwdArgs& m, float* work, int64_t work_floats, int max_slabs, int* nslab,
                    hipStream_t stream, int phase = 0, int t_lo = 0, int t_hi = 0, float* ghw_carry = nullptr);
int64_t mixer_split_work_floats(const t2o_layout& L, int B, int T);
bool mixer_split_taken(const t2o_layout& L, int B);
int mixer_split_extra_slabs(int B);
// Launch shape of a one-wave-per-episode mixer kernel: weights staged in LDS (wfl
// floats) beside wmax_lds .. min_lds per-wave buffers (perw floats, halving), else
// read through L2 beside wmax_l2 .. min_l2 buffers alone; waves = 0 when neither
// fits.  LDS weights first: the placement every parity test ran.  (fp32 at 16 AGVs:
// 121 KB of weights leave room for two waves per CU, half the SIMDs idle — DESIGN §9
// item 4 for the L2 alternative, not measured.)
struct MixLaunch {
  int waves;
  bool wlds;
  size_t lds;  // bytes
};
inline MixLaunch mix_pick(size_t wfl, size_t perw, int wmax_lds, int min_lds, int wmax_l2, int min_l2) {
  constexpr size_t CAP = 160 * 1024;
  MixLaunch m{};
  for (m.waves = wmax_lds, m.wlds = true; m.waves >= min_lds; m.waves >>= 1) {
    m.lds = sizeof(float) * (wfl + (size_t)m.waves * perw);
    if (m.lds <= CAP) return m;
  }
  for (m.waves = wmax_l2, m.wlds = false; m.waves >= min_l2; m.waves >>= 1) {
    m.lds = sizeof(float) * (size_t)m.waves * perw;
    if (m.lds <= CAP) return m;
  }
  return MixLaunch{0, false, 0};
}

}  // namespace t2o
