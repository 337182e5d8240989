/*
 * t2omca.h — C-ABI of the MI355X-native T2OMCA learner hot path.
 *
 * The reference (hj5717/T2OMCA) is pure Python/PyTorch; its "plugin API" for
 * this path is two nn.Module classes driven by PyMARL registries
 * (SURVEY.md §8 b).  Every entry point below replaces one piece of the
 * reference's CPU arithmetic and is bound from Python with ctypes
 * (t2omca_amd/_lib.py; see INTEGRATION.md for the binding a maintainer adds
 * to the reference tree):
 *
 *   t2o_agent_unroll_fwd   TransformerAgent.forward unrolled over t
 *                          (transf_agent.py:54-76, transformer.py:40-178)
 *   t2o_agent_unroll_bwd   BPTT of the above (autograd of the same lines)
 *   t2o_mixer_unroll_fwd   TransformerMixer.forward unrolled over t
 *                          (n_transf_mixer.py:55-91) incl. the learner's
 *                          chosen-Q gather / double-Q argmax
 *   t2o_mixer_unroll_bwd   BPTT of the above
 *   t2o_td_loss            learner.train's TD target / loss / priorities
 *                          (call site per_run.py:224-238; PyMARL2 contract)
 *   t2o_adam_step          optimiser step with global-norm clipping
 *   t2o_env_step / reset   MultiAgvOffloadingEnv.step/reset/get_obs/get_state
 *                          (environment_multi_mec.py:184-366, normalization.py)
 *
 * Conventions (all entry points):
 *   - arguments are raw device pointers + explicit sizes + a hipStream_t
 *     passed as void*; the library never allocates or frees device memory and
 *     never synchronises: the caller owns every buffer, including workspaces;
 *   - return 0 on success, a negative T2O_E* code on a bad argument, or the
 *     positive hipError_t of a failed launch;
 *   - float tensors are fp32, row-major, contiguous unless a stride is given.
 */
#ifndef T2OMCA_H
#define T2OMCA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define T2O_MAX_DEPTH 4

/* Bumped whenever an entry point's signature, t2o_layout, or a workspace / tape
 * size or layout formula changes, so a binding built against one header can
 * refuse a library built from another (t2o_abi_version).  History: 3 = round-3
 * library (tuned one-tile mixers write one compact tape stream per block,
 * ceil(B*T*(A+3)/16) tiles; records of 4E + 2HE features); 4 = t2o_td_loss_ex2,
 * t2o_bwd_tape_contract_pair, t2o_abi_version; 5 = the step-range / split-phase
 * entry points; 6 = one argument struct per unroll / BPTT / contraction / TD
 * loss entry point (their _ex / _ex2 / _range / _split / _pair generations
 * folded in), t2o_args_sizeof, t2o_agent_bwd_ranges. */
#define T2O_ABI_VERSION 6
int t2o_abi_version(void);

enum {
  T2O_OK = 0,
  T2O_EINVAL = -1,      /* unsupported size / null pointer */
  T2O_EUNSUPPORTED = -2 /* no kernel instantiated for this (E, H, D, n) */
};

/* Offsets (in elements) of every tensor of one network's device pack.  The pack
 * holds the folded weights the kernels read (M_h = Wk_hᵀWq_h/√E,
 * N_h = U_h·Wv_h, zero-padded embedding / head matrices) plus transposed
 * copies for the backward.  Order: forward matrices [0, vec_lo), forward
 * vectors (biases, LayerNorm) [vec_lo, fwd_total), transposed copies
 * [fwd_total, total).  kind 0 = agent, 1 = mixer.
 * prec 0 (fp32): the pack is `total` floats.  prec 1 (bf16 MFMA operands): the
 * fp32 pack is followed, at float offset `total`, by a bf16 image of it (the
 * kernels read matrices from the image and vectors from the fp32 part); the
 * buffer is `pack_floats` floats.  Activations, LayerNorm, softmax, recurrent
 * state and every accumulation stay fp32 in both modes. */
typedef struct {
  int32_t kind, E, H, D, F, NA, FF, n_ent;
  int32_t prec;
  int32_t generic;            /* 1: no tuned kernel instance for this shape; the
                                 runtime-shaped kernels run (t2o_generic.hip) and the
                                 pack is the reference-order parameters followed by
                                 transposed copies; compact grads = reference order */
  int64_t WeT, We, be;        /* WeT[16][E], We[E][16], be[E] (F <= 16) */
  int64_t Wo, bo, WoT;        /* agent: q_basic padded Wo[16][E], bo[16], WoT[E][16];
                                 mixer: hyper_b2.weight in Wo row 0, bias in bo[0] */
  int64_t M[T2O_MAX_DEPTH], MT[T2O_MAX_DEPTH];   /* [H*E][E], [E][H*E] */
  int64_t N[T2O_MAX_DEPTH], NT[T2O_MAX_DEPTH];   /* [E][H*E], [H*E][E] */
  int64_t bu[T2O_MAX_DEPTH], g1[T2O_MAX_DEPTH], n1[T2O_MAX_DEPTH];
  int64_t W1[T2O_MAX_DEPTH], W1T[T2O_MAX_DEPTH], c1[T2O_MAX_DEPTH]; /* [FF][E],[E][FF],[FF] */
  int64_t W2[T2O_MAX_DEPTH], W2T[T2O_MAX_DEPTH], c2[T2O_MAX_DEPTH]; /* [E][FF],[FF][E],[E] */
  int64_t g2[T2O_MAX_DEPTH], n2[T2O_MAX_DEPTH];
  int64_t fwd_total;          /* elements [0, fwd_total) = every tensor the forward reads */
  int64_t total;              /* elements of the pack */
  int64_t grad_total;         /* size of the compact gradient block (no transposes) */
  int64_t vec_lo;             /* first vector element (see above) */
  int64_t pack_floats;        /* buffer size of a pack in floats (prec 1: fp32 + bf16 image) */
  int32_t n_agents;           /* mixer: agents (hidden tokens, qvals, w1 rows); n_ent = its state
                                 tokens (n_entities_state, or n_agents * n_entities for the obs
                                 branch of n_transf_mixer.py:62-63).  agent: = n_ent */
  int32_t pos_func;           /* mixer head positivity (n_transf_mixer.py:95-103):
                                 T2O_POS_ABS / _SOFTPLUS / _QUADRATIC / _IDENTITY */
  float pos_beta;             /* softplus beta (qmix_pos_func_beta) */
  int32_t reserved_;
} t2o_layout;

#define T2O_POS_ABS 0
#define T2O_POS_SOFTPLUS 1
#define T2O_POS_QUADRATIC 2
#define T2O_POS_IDENTITY 3

/* t2o_layout_init_ex flags */
#define T2O_LAYOUT_FORCE_GENERIC 1  /* use the runtime-shaped kernels even for a tuned shape */

/* Fill *L for a network (prec 0 = fp32, 1 = bf16 MFMA operands); returns 0 or T2O_EINVAL.
 * Shapes with a tuned MFMA kernel instance get the folded MFMA pack: the default
 * network (E 32 / 3 heads / depth 2 / FF 128) at any entity count 1..64 — exact
 * instances at 3, 8, 16 and 64, runtime-entity instances of capacity 8 / 16 / 64
 * (agent) and 8 / 13 / 16 / 32 / 64 (mixer) otherwise (t2o_layout_instance) — and
 * E 16 / 2 heads / depth 1 / FF 64 at 3 (a fixture shape).  Any other shape within
 * the runtime-shaped kernels' limits (E <= 64, H <= 8, H*E <= 512, D <= 4, FF <= 512,
 * F <= 16, NA <= 16, agent entities <= 64, mixer tokens n_ent + n_agents + 3 <= 192
 * with n_agents <= 64), a mixer head other than abs, or n_agents != n_ent, gets
 * generic = 1.  The generic kernels compute in fp32 whatever prec says. */
int t2o_layout_init(t2o_layout* L, int kind, int E, int H, int D, int F, int NA, int FF, int n_ent, int prec);
/* t2o_layout_init with the mixer's agent count (n_agents; 0 = n_ent), its head's
 * positivity function (T2O_POS_*, softplus beta) and flags (T2O_LAYOUT_*). */
int t2o_layout_init_ex(t2o_layout* L, int kind, int E, int H, int D, int F, int NA, int FF, int n_ent, int prec,
                       int n_agents, int pos_func, float pos_beta, int flags);

/* Which kernels a layout runs: T2O_INSTANCE_EXACT (MFMA instance compiled for its
 * entity count), T2O_INSTANCE_RUNTIME (MFMA instance of a capacity class, entity
 * count read at run time), T2O_INSTANCE_GENERIC (runtime-shaped fp32 kernels);
 * negative on a null layout. */
#define T2O_INSTANCE_EXACT 0
#define T2O_INSTANCE_RUNTIME 1
#define T2O_INSTANCE_GENERIC 2
int t2o_layout_instance(const t2o_layout* L);

/* sizeof(t2o_layout), for bindings to check their mirror of the struct. */
int t2o_layout_sizeof(void);

/* Reference parameter order (state_dict order of transf_agent.py /
 * n_transf_mixer.py, SURVEY.md §8 b) flattened into one fp32 buffer:
 *   feat_embedding.{weight[E][F], bias[E]},
 *   per block: tokeys[HE][E], toqueries[HE][E], tovalues[HE][E],
 *              unifyheads.{weight[E][HE], bias[E]}, norm1.{w,b}[E], norm2.{w,b}[E],
 *              ff.0.{weight[FF][E], bias[FF]}, ff.2.{weight[E][FF], bias[E]},
 *   agent: q_basic.{weight[NA][E], bias[NA]};  mixer: hyper_b2.{weight[1][E], bias[1]}.
 * Returns the number of floats. */
int64_t t2o_param_count(int kind, int E, int H, int D, int F, int NA, int FF);

/* params (reference order) -> device pack (folded + padded + transposed). */
int t2o_pack_params(const t2o_layout* L, const float* params, float* pack, void* stream);

/* compact gradient block (pack layout, from the backward kernels) ->
 * gradients in the reference parameter order (accumulated: grad += ...). */
int t2o_unpack_grads(const t2o_layout* L, const float* params, const float* gpack,
                     float* grad, void* stream);

/* ---- The unrolls, their BPTTs, the tape contraction and the TD loss take ONE
 * argument struct each (ABI 6): named fields instead of 25-45 positional
 * arguments, so a binding cannot shift a pointer into the wrong slot unnoticed.
 * Bindings check their mirror of every struct with t2o_args_sizeof. */
#define T2O_ARGS_AGENT_FWD 0
#define T2O_ARGS_AGENT_BWD 1
#define T2O_ARGS_MIXER_FWD 2
#define T2O_ARGS_MIXER_BWD 3
#define T2O_ARGS_TAPE 4
#define T2O_ARGS_TD 5
int t2o_args_sizeof(int which); /* sizeof the T2O_ARGS_* struct, -1 for an unknown one */

/* Agent unroll forward (TransformerAgent.forward over t, transf_agent.py:54-76) for
 * up to two networks sharing the observations (online + target). */
typedef struct {
  const t2o_layout* L;
  const float* pack_on;
  const float* pack_tg;       /* NULL: one network (q_tg / h_tg / hmid_tg unused) */
  const float* obs;           /* [b][t][a][n_ent*F], element strides obs_sb, obs_st */
  int64_t obs_sb, obs_st;
  const float* h0_on;         /* [B][A][E]; NULL = zeros (init_hidden) */
  const float* h0_tg;
  float* q_on;                /* out [b][t][a][NA] */
  float* h_on;                /* out [b][t][a][E]: h after step t */
  float* hmid_on;             /* out [b][t][D-1][a][E] block inputs (NULL: not kept) */
  float* q_tg;
  float* h_tg;
  float* hmid_tg;
  int32_t B, T, A;
  int32_t t0, t1;             /* steps [t0, t1) of T (t1 <= 0: T); t0 > 0 continues from h at t0 - 1
                                 (what the range before wrote; outputs are indexed by the full T) */
} t2o_agent_fwd_args;
int t2o_agent_unroll_fwd(const t2o_agent_fwd_args* a, void* stream);

/* Agent BPTT of one network over steps t_hi - 1 .. t_lo (default: T - 1 .. 0). */
typedef struct {
  const t2o_layout* L;
  const float* pack;
  const float* obs;           /* as the forward's */
  int64_t obs_sb, obs_st;
  const float* h0;            /* as the forward's (NULL = zeros) */
  const float* h_seq;         /* forward h [b][h_ts][a][E], h_ts >= T */
  const float* hmid;          /* forward hmid [b][h_ts][D-1][a][E] or NULL (recomputed) */
  int32_t h_ts;
  const float* gq;            /* dL/dq [b][t][a][NA] or NULL */
  const float* gchosen;       /* dL/dq[action] [b][t][a] or NULL (needs actions) */
  const int64_t* actions;     /* [b][t][a], element strides act_sb, act_st, a-stride 1 */
  int64_t act_sb, act_st;
  const float* gh;            /* dL/dh [b][t][a][E] or NULL */
  float* gslabs;              /* out [nslab][grad_total] per-workgroup partial gradients (compact
                                 layout, overwritten); complete after t2o_bwd_tape_contract */
  int32_t max_slabs;          /* >= t2o_agent_bwd_max_slabs(B, A) */
  int32_t* nslab;             /* out: slabs written */
  void* tape;                 /* workspace t2o_bwd_tape_floats(L, t2o_bwd_tape_tiles(L, B, T, A)) floats */
  float* gh0;                 /* out dL/dh0 [B][A][E] or NULL */
  float* gcarry;              /* [B*A][E] dL/dh between step ranges (read at t_hi < T, written at t_lo > 0) */
  int32_t B, T, A;
  int32_t t_lo, t_hi;         /* t_hi <= 0: T.  A partial range needs the pipelined BPTT
                                 (t2o_agent_bwd_ranges; else T2O_EUNSUPPORTED); ranges run from the
                                 last one down on the same slabs (the first clears them) and tape */
} t2o_agent_bwd_args;
int t2o_agent_unroll_bwd(const t2o_agent_bwd_args* a, void* stream);
int t2o_agent_bwd_max_slabs(int B, int A);
/* The record format t2o_agent_unroll_bwd writes to its tape for this layout
 * (has_hmid: the call passes hmid): 0 the full record; 1 (bf16, the pipelined
 * kernel, up to 8 entities) the lean record — dM and dN were accumulated in
 * registers and flushed into the slabs, the tape holds only the FFN / LN1 /
 * unify-bias operands.  Pass it to the contraction (t2o_tape_args.rec_format). */
int t2o_agent_bwd_tape_format(const t2o_layout* L, int has_hmid);
/* 1 when t2o_agent_unroll_bwd accepts a partial step range for this layout
 * (has_hmid: the call passes hmid): the two-wave pipelined BPTT runs it (depth 2,
 * its LDS fits, T2O_AGENT_BWD is not "single").  Otherwise 0, and the one-wave
 * kernel takes only the whole unroll (a partial range returns T2O_EUNSUPPORTED).
 * The learner's pipelined update (step ranges on two streams) asks this first. */
int t2o_agent_bwd_ranges(const t2o_layout* L, int has_hmid);

/* Mixer unroll forward (TransformerMixer.forward over t, n_transf_mixer.py:55-91)
 * for up to two networks (online + target) in one launch, with the learner's
 * chosen-Q gather / double-Q argmax.  qmode: 0 = qvals given (qv_* [B][T][A]);
 * 1 = chosen-action gather from the network's Q array (q_on / q_tg
 * [b][q_ts][a][n_actions] at actions); 2 = double-Q: the network's Q array at
 * argmax_a' of q_on masked by avail (NULL = all available), ties -> lowest index. */
typedef struct {
  const t2o_layout* L;
  const float* pack_on;
  const float* pack_tg;       /* NULL: one network */
  const float* states;        /* [b][t][n_ent*F], element strides st_sb, st_st */
  int64_t st_sb, st_st;
  const float* hid_on;        /* agent hidden states [b][t][a][E], strides hid_sb, hid_st, a-stride E */
  const float* hid_tg;
  int64_t hid_sb, hid_st;
  const float* hw0_on;        /* initial hyper tokens [B][3][E]; NULL = zeros */
  const float* hw0_tg;
  int32_t qmode_on, qmode_tg;
  const float* qv_on;
  const float* qv_tg;
  const float* q_on;
  const float* q_tg;
  int32_t q_ts, n_actions;
  const int64_t* actions;     /* [b][t][a], strides act_sb, act_st */
  int64_t act_sb, act_st;
  const int32_t* avail;       /* [b][t][a][n_actions], strides av_sb, av_st, or NULL */
  int64_t av_sb, av_st;
  float* y_on;                /* out [B][T] */
  float* hw_on;               /* out [B][T][3][E] hyper tokens after step t */
  float* qvo_on;              /* out [B][T][A] qvals used, or NULL */
  float* xout_on;             /* out [B][T][A+3][E] final query rows, or NULL (the backward needs them,
                                 and a decoupled multi-tile mixer needs them for every network) */
  float* xmid_on;             /* out [B][T][D-1][A+3][E] block inputs, or NULL (recomputed) */
  float* y_tg;
  float* hw_tg;
  float* qvo_tg;
  float* xout_tg;
  float* xmid_tg;
  int32_t B, T_on, T_tg;
  int32_t phase;              /* 0: the whole unroll.  A decoupled mixer (t2o_mixer_split) may run its
                                 phases beside the agent's step ranges on another stream: 1 = the
                                 recurrence over steps [t0, t1) (the window's rows, hw, their xout /
                                 xmid), every range in order; then 2 = every (episode, step)'s other
                                 rows and the mixing head.  T2O_EUNSUPPORTED when it does not run
                                 decoupled. */
  int32_t t0, t1;
} t2o_mixer_fwd_args;
int t2o_mixer_unroll_fwd(const t2o_mixer_fwd_args* a, void* stream);

/* Mixer BPTT of one network over steps T-1..0. */
typedef struct {
  const t2o_layout* L;
  const float* pack;
  const float* states;
  int64_t st_sb, st_st;
  const float* hid;
  int64_t hid_sb, hid_st;
  const float* hw0;
  const float* qv;            /* forward qvo [B][T][A] */
  const float* hw;            /* forward hw */
  const float* xout;          /* forward xout (required) */
  const float* xmid;          /* forward xmid or NULL */
  const float* gy;            /* dL/dy [B][T] */
  const float* ghw_ext;       /* extra dL/dhw [B][T][3][E] or NULL */
  float* gqv;                 /* out dL/dqvals [B][T][A] */
  float* ghid;                /* out dL/dhidden states [B][T][A][E] */
  float* ghw0;                /* out dL/dhw0 [B][3][E] or NULL */
  float* gslabs;              /* out partial weight-grad slabs, as the agent's */
  int32_t max_slabs;          /* >= t2o_mixer_bwd_max_slabs(B) */
  int32_t* nslab;
  void* tape;                 /* t2o_bwd_tape_floats(L, tiles) floats, tiles = t2o_bwd_tape_tiles(L, B, T, A) */
  float* work;                /* t2o_mixer_bwd_work_floats(L, B, T) floats, or NULL: lets a multi-tile
                                 mixer (A + 3 > 16 query rows) at a small batch run its recurrence
                                 decoupled (the window of the last 16 query rows carries the hyper
                                 tokens, every (episode, step)'s other rows run in parallel; the key
                                 gradients sum in another order) */
  int64_t work_floats;
  float* ghw_carry;           /* [B][3][E] hyper grads between phase-2 step ranges */
  int32_t B, T;
  int32_t phase;              /* 0: the whole BPTT; decoupled: 1 = every (episode, step)'s parallel part,
                                 then 2 = the recurrence over steps t_hi - 1 .. t_lo, ranges from the
                                 last one down (*nslab the same for every call) */
  int32_t t_lo, t_hi;         /* t_hi <= 0: T */
} t2o_mixer_bwd_args;
int t2o_mixer_unroll_bwd(const t2o_mixer_bwd_args* a, void* stream);
int t2o_mixer_bwd_max_slabs(int B);
/* Workspace floats t2o_mixer_unroll_bwd can use for this layout and batch
 * (0: the layout has one query tile, nothing to decouple; -1 bad argument). */
int64_t t2o_mixer_bwd_work_floats(const t2o_layout* L, int B, int T);
/* 1 when a mixer of this layout runs decoupled at batch B (forward: when every
 * network's xout is given; backward: with the workspace), else 0.
 * T2O_MIXER_SPLIT=0 / 1 in the environment forces it off / on. */
int t2o_mixer_split(const t2o_layout* L, int B);

/* Tiles of 16 weight-gradient records per block that one backward call writes
 * (agent: T * ceil(B*A/16); mixer, A = L->n_agents: B*T*ceil((A+3)/16), or for
 * a tuned mixer with A+3 > 16 query rows, whose records form one compact stream
 * per block, ceil(B*T*(A+3)/16)).  -1 on a bad argument.  Both the tape size
 * (t2o_bwd_tape_floats) and the contraction's `tiles` take this count. */
int64_t t2o_bwd_tape_tiles(const t2o_layout* L, int B, int T, int A);

/* Floats of backward tape workspace for `tiles` tiles of 16 records:
 * D * tiles * 16 * (4E + 2HE) elements of 4 (fp32) or 2 (bf16) bytes. */
int64_t t2o_bwd_tape_floats(const t2o_layout* L, int64_t tiles);

/* One backward call's weight-gradient tape, to be contracted into its slabs. */
typedef struct {
  const t2o_layout* L;
  const float* pack;          /* the kernel pack the backward used (g1, n1, W1, W2ᵀ, c1 recompute the
                                 FFN operands the tape does not store) */
  const void* tape;
  int64_t tiles;              /* the backward's t2o_bwd_tape_tiles (the tape's per-block stride) */
  float* gslabs;              /* the backward's slabs */
  int32_t nslab;              /* >= the backward's *nslab: slabs past it must be zeroed by the caller
                                 (a small batch's contraction over more workgroups) */
  int32_t rec_format;         /* t2o_agent_bwd_tape_format; 0 = the full record (every mixer's) */
} t2o_tape_args;
/* Contract a backward tape (dM, dN, dW2, P = Σ_records dYᵀ X, split-K over the
 * slabs) into the M/N/W1/W2 regions of its slabs.  The W1 / g1 regions then hold
 * P = Σ gf1 ⊗ x̂1 and Q = Σ gr2 ⊙ x̂1, which t2o_unpack_grads turns into the W1 /
 * norm1 grads.  Format 1 adds only the FFN / LN1 / bu grads (the backward put dM /
 * dN into the slabs).  With `second` (or NULL): BOTH backwards' tapes in one
 * launch — `first` the mixer's (format 0), `second` the agent's — each exactly as
 * alone, one grid of both slab counts (the two share the chip from the start);
 * layouts that are not tuned instances of one network shape and precision run as
 * two launches.  Must follow the t2o_*_unroll_bwd call(s) on the same stream. */
int t2o_bwd_tape_contract(const t2o_tape_args* first, const t2o_tape_args* second, void* stream);

/* Element types of the TD loss's mask inputs. */
#define T2O_DT_F32 0
#define T2O_DT_U8 1   /* uint8 / bool: EpisodeBatch "terminated" */
#define T2O_DT_I32 2
#define T2O_DT_I64 3  /* int64: EpisodeBatch "filled" */

/* TD loss algorithms */
#define T2O_TD_AUTO 0        /* the library's default (currently T2O_TD_WAVE_SCAN, the faster) */
#define T2O_TD_SEQUENTIAL 1  /* one thread per episode, the reference's backward order (T <= ~4900) */
#define T2O_TD_WAVE_SCAN 2   /* one wave per episode: suffix scan of the linear TD(λ) recursion
                                (reassociated: fp32 rounding differs by ~1e-7 relative; any T) */

/* TD(λ) targets, masked PER-weighted loss, dL/dQtot and priorities (PyMARL2
 * NQLearner semantics, learner.train at per_run.py:224-238; t2o_learner.hip). */
typedef struct {
  const float* qtot;          /* [B][T] online mixer */
  const float* qtot_tgt;      /* [B][T+1] target mixer */
  const float* reward;        /* [b][t], element strides rw_sb, rw_st */
  int64_t rw_sb, rw_st;
  const void* term;           /* [b][t] 0/1 (NULL: none), element type term_dtype, strides tm_* */
  int64_t tm_sb, tm_st;
  const void* filled;         /* [b][t] 0/1 (NULL: all), element type filled_dtype, strides fl_* */
  int64_t fl_sb, fl_st;
  const float* per_weight;    /* [B] or NULL (= 1) */
  float* gq;                  /* out [B][T] dL/dQtot */
  float* targets;             /* out [B][T] or NULL */
  float* prio;                /* out [B] */
  float* loss;                /* out [2] = {loss, local Σ mask} */
  float* mask_sum_acc;        /* NULL, or += local Σ mask (the learner keeps Σ mask in its flat
                                 gradient's last slot: the data-parallel all-reduce sums it with the
                                 grads and Adam divides by the global value) */
  float gamma, td_lambda;
  float mask_sum;             /* > 0: normalise gq / loss by this global Σ mask; else by the local one */
  int32_t term_dtype, filled_dtype;  /* T2O_DT_*: the EpisodeBatch's own types, read in place */
  int32_t algo;               /* T2O_TD_* */
  int32_t B, T;
} t2o_td_args;
int t2o_td_loss(const t2o_td_args* a, void* stream);

/* clip_grad_norm_(max_grad_norm) + Adam (torch.optim.Adam semantics, L2
 * weight decay) over n floats.  workspace: t2o_adam_workspace_floats() floats
 * (needed when max_grad_norm > 0).  grad_div [1] (may be NULL): device scalar
 * every grad is divided by first (the global Σ mask under data parallelism).
 * grad_norm_out [1] may be NULL. */
int t2o_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                  float* workspace, int64_t n, double lr, double beta1, double beta2, float eps,
                  float weight_decay, float max_grad_norm, int64_t step, const float* grad_div,
                  float* grad_norm_out, void* stream);
int t2o_adam_workspace_floats(void);

/* Diagnostic: runs the cross-lane primitives the kernels rely on (4-lane
 * all-reduces via ds_bpermute and via gfx950 permlane swaps, 16-lane DPP row
 * sums, the batched all-reduce) on in[64]; writes 20 x 64 results
 * (tests/test_gpu_primitives.py). */
int t2o_probe_lane_ops(const float* in, float* out, void* stream);

/* Diagnostic: the mixing head's positivity function pos_func (T2O_POS_*,
 * n_transf_mixer.py:95-103) with beta on x[n]: out[0:n] posf, out[n:2n] its
 * derivative, out[2n:4n] the fused value / derivative pair the BPTT kernels
 * evaluate (tests/test_gpu_primitives.py checks them element by element). */
int t2o_probe_posf(const float* x, int n, int pos_func, float beta, float* out, void* stream);

/* Diagnostic: the agent softmax's reduce-scatter / broadcast halves of the batched
 * 4-lane all-reduce, the packed 4-feature dot product and the 8-wide bf16
 * conversion with the bit-pattern ReLU, on in[64]; writes 23 x 64 results
 * (tests/test_gpu_primitives.py). */
int t2o_probe_scatter_ops(const float* in, float* out, void* stream);
/* Diagnostic: MFMA result hand-offs after a fixed number of wait states (inline
 * asm, unpadded by the compiler): a 16x16x4 f32 result stored to LDS / global
 * memory from its AGPRs after 10 or 32 states, a 16x16x32 bf16 result read as
 * srcC by a 16x16x16 bf16 MFMA after 0 / 4 / 32 states and by a 16x16x32 after
 * 0 / 32, then the compiler-built references.  in [nwaves][64][12] floats, out
 * [12][nwaves][64][4] floats (t2o_probe.hip). */
int t2o_probe_xdl_hazards(const float* in, float* out, int nwaves, void* stream);

/* Diagnostic: the XOR (in bf16 elements, a multiple of 8) applied to the
 * columns of row `row` of a bf16 weight-image matrix with row length ld: element
 * (r, col) of the image sits at r*ld + (col ^ t2o_bf_swz(r, ld)). */
int t2o_bf_swz(int row, int ld);

/* Sum nslab partial gradient slabs [nslab][n] into out[n] (out = sum, overwritten). */
int t2o_reduce_slabs(const float* slabs, int nslab, int64_t n, float* out, void* stream);

/* ---- vectorised MEC-offloading environment -------------
 * Replaces MultiAgvOffloadingEnv (environment_multi_mec.py:12-439) driven by
 * parallel_runner.py's env_worker (:224-270): NE envs advance in lock-step, one
 * wave per env, state resident in HBM.  All arrays but spec are device pointers.
 *
 * mode 0  construction (:12-59: mec_index + positions, zeroed queues/normaliser)
 * mode 1  worker 'reset'  (:257-263 -> reset() :219-227, get_state, get_avail_actions, get_obs)
 * mode 2  worker 'step'   (:239-256 -> step() :309-366, get_state, get_avail_actions, get_obs)
 * mode 3  get_env_info's two get_obs calls (:421-439; normaliser updates only)
 *
 * spec[15] (fp64, host memory): mec_radius, computation_cycles, bandwidth, noise_power,
 *   path_loss, channel_gain_linear, mec_compute_cap, agv_transmit_power,
 *   agv_compute_cap, latency_max, t_length, job_size_min, job_size_max,
 *   job_arrival_p, edge_only (0/1)  (t2omca_amd/env_spec.py).  Entity
 *   observations (obs_entity_mode = True).
 * state[17]: mec_index i32[NE][A], x f64[NE][A], y f64[NE][A],
 *   q_size i32[NE][A][QMAX], q_thr i32[NE][A][QMAX], q_head i32[NE][A],
 *   q_len i32[NE][A], task_num i32[NE][A], task_success i32[NE][A],
 *   remain_delay f64[NE][A], last_ack i32[NE][A], time_slot i32[NE],
 *   draw i64[NE], nrm_n i64[NE], nrm_mean f64[NE][9A], nrm_S f64[NE][9A],
 *   nrm_std f64[NE][9A].
 * out[8] (any entry may be NULL except reward/terminated/info in mode 2):
 *   obs f32[NE][A][9A], obs f64[NE][A][9A], state f32[NE][8A],
 *   avail i32[NE][A][C+1], reward f64[NE], terminated u8[NE],
 *   info f64[NE][6] = delay_reward, overtime_penalty, channel_utilization_rate,
 *   conflict_ratio, task_completion_rate, task_completion_delay (NaN unless terminal),
 *   ack i32[NE][A].
 * actions: i64, env e's agent a at actions[e*act_se + a] (values in 0..C).
 * Limits: A <= 64, M <= 16, C <= 16.  Random draws: env_spec.uniforms(seed, env, draw). */
int t2o_env_run(int mode, const double* spec, void* const* state, void* const* out,
                const int64_t* actions, int64_t act_se, int NE, int A, int M, int C, int QMAX, int T,
                uint64_t seed, void* stream);

/* t2o_env_run with spec[16] (host memory): spec[15] = obs_entity_mode (1: the
 * entity observation [A][9A] above; 0: get_obs_agent's flat branch, :172-182,
 * obs f32/f64[NE][A][6] = [last_ack, get_agent_inf], normalised by the env's
 * 6-long running normaliser, which keeps its [9A] row stride in state[14..16]),
 * and n_out = 8 (as above) or 11 output pointers; the extra three
 * carry the compact observation wire format (replaces storing
 * get_obs's dense [A][9A] output, environment_multi_mec.py:148-186):
 *   out[8]  wire i32[NE][A][4], written with every obs the worker returns
 *           (modes 1, 2): per entity j, w0 = job size, w1 = data_delay,
 *           w2 = offload delay x 100 (exact integer: the fp64 value is
 *           rint(x*100)/100), w3 = thr | qlen << 16 | (ack+1) << 24 | mec << 26;
 *           all zero fields when the queue is empty (get_agent_inf :123-146);
 *   out[9]  snap_n i64[NE], out[10] snap f64[NE][2][9A]: the normaliser's
 *           count, mean and S right before the worker's get_obs in mode 1 (the
 *           state the episode's first returned obs is normalised from).
 * out[9] / out[10] are both set or both NULL.  Needs latency_max <= 65535.
 * The wire format needs entity observations (spec[15] = 1). */
int t2o_env_run_ex(int mode, const double* spec, void* const* state, void* const* out, int n_out,
                   const int64_t* actions, int64_t act_se, int NE, int A, int M, int C, int QMAX, int T,
                   uint64_t seed, void* stream);

/* Dense normalised observations from the wire format: for each episode b,
 * starting from (snap_n[b], snap[b]), replays get_obs's sequential normaliser
 * (normalization.py:12-35, agent by agent, t = 0..T1-1) on the observation
 * get_obs_agent (:148-182) builds from wire[b][t] — bit-identical to the env's
 * own obs output.  wire: int32 element strides w_sb / w_st (multiples of 4,
 * 16-B aligned), rows [A][4] dense; obs: f32 element strides o_sb / o_st, each
 * step a dense [A][9A]; obs64 (optional) dense f64 [B][T1][A][9A].  A <= 64. */
int t2o_obs_expand(const int32_t* wire, int64_t w_sb, int64_t w_st, const int64_t* snap_n, const double* snap,
                   float* obs, int64_t o_sb, int64_t o_st, double* obs64, int B, int T1, int A, void* stream);

/* ε-greedy action selection (the reference's controller is
 * absent, contract parallel_runner.py:121 with PyMARL's EpsilonGreedyActionSelector).
 * q f32 [rows][NA], avail i32 [rows][NA] (rows = envs x agents, dense) ->
 * actions i64 [rows]: argmax of q over available actions (first maximum), or
 * with probability epsilon a uniformly drawn available action.  Draws:
 * u1 = U(seed, row, 2*counter), u2 = U(seed, row, 2*counter+1) of the
 * env_spec.uniforms stream; random action = floor(u2 * n_avail)-th available.
 * NA <= 32. */
int t2o_select_actions(const float* q, const int32_t* avail, int64_t* actions, int64_t rows, int NA,
                       double epsilon, uint64_t seed, int64_t counter, void* stream);

/* Prioritized episode replay (the reference's buffer is
 * absent, contract per_run.py:143-146,216-238, PyMARL2 proportional PER).
 * p f32 [n] = stored priority**alpha of the n valid episodes.  Sample batch
 * indices by stratified proportional search (mass_k = (u_k + k) * Σp / batch,
 * u_k = U(seed, k, counter)) with IS weights (p_i/Σp*n)^-beta normalised by
 * the weight of min p; workspace: t2o_per_workspace_doubles(n) doubles. */
int64_t t2o_per_workspace_doubles(int64_t capacity);
int t2o_per_sample(const float* p, int64_t n, int64_t batch, double beta, uint64_t seed, int64_t counter,
                   double* workspace, int64_t* idx_out, float* w_out, void* stream);
/* p[idx[k]] = (prio[k] + eps)**alpha; *max_prio = max(*max_prio, prio[k] + eps). */
int t2o_per_update(float* p, const int64_t* idx, const float* prio, int64_t n, float alpha, float eps,
                   float* max_prio, void* stream);
/* dst + k*dst_stride <- src + idx[k]*src_stride, row_bytes each (rows <= 65535;
 * copied in the widest of 16/8/4/1-byte units the alignment allows): the
 * episode gather of a sampled batch. */
int t2o_gather_rows(const void* src, int64_t src_stride, const int64_t* idx, int64_t rows, void* dst,
                    int64_t dst_stride, int64_t row_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* T2OMCA_H */
