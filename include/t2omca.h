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

enum {
  T2O_OK = 0,
  T2O_EINVAL = -1,      /* unsupported size / null pointer */
  T2O_EUNSUPPORTED = -2 /* no kernel instantiated for this (E, H, D, n) */
};

/* Offsets (in floats) of every tensor of one network's device pack.  The pack
 * holds the folded weights the kernels read (M_h = Wk_hᵀWq_h/√E,
 * N_h = U_h·Wv_h, zero-padded embedding / head matrices) plus transposed
 * copies for the backward.  A gradient slab uses the same layout; its
 * transposed entries are unused.  kind 0 = agent, 1 = mixer. */
typedef struct {
  int32_t kind, E, H, D, F, NA, FF, n_ent;
  int64_t WeT, We, be;        /* WeT[16][E], We[E][16], be[E] (F <= 16) */
  int64_t Wo, bo, WoT;        /* agent: q_basic padded Wo[16][E], bo[16], WoT[E][16];
                                 mixer: hyper_b2.weight in Wo row 0, bias in bo[0] */
  int64_t M[T2O_MAX_DEPTH], MT[T2O_MAX_DEPTH];   /* [H*E][E], [E][H*E] */
  int64_t N[T2O_MAX_DEPTH], NT[T2O_MAX_DEPTH];   /* [E][H*E], [H*E][E] */
  int64_t bu[T2O_MAX_DEPTH], g1[T2O_MAX_DEPTH], n1[T2O_MAX_DEPTH];
  int64_t W1[T2O_MAX_DEPTH], W1T[T2O_MAX_DEPTH], c1[T2O_MAX_DEPTH]; /* [FF][E],[E][FF],[FF] */
  int64_t W2[T2O_MAX_DEPTH], W2T[T2O_MAX_DEPTH], c2[T2O_MAX_DEPTH]; /* [E][FF],[FF][E],[E] */
  int64_t g2[T2O_MAX_DEPTH], n2[T2O_MAX_DEPTH];
  int64_t total;              /* pack size in floats */
  int64_t grad_total;         /* size of the compact gradient block (no transposes) */
} t2o_layout;

/* Fill *L for a network; returns 0 or T2O_EINVAL. */
int t2o_layout_init(t2o_layout* L, int kind, int E, int H, int D, int F, int NA, int FF, int n_ent);

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

/* Agent unroll forward over T steps for up to two networks sharing the
 * observations (online + target).  obs[b][t][a][n_ent*F] with element strides
 * obs_sb, obs_st (a-stride = n_ent*F).  h0 may be NULL (zeros, init_hidden).
 * Outputs q[b][t][a][NA], h[b][t][a][E] (h after step t).  pack_tg/q_tg/h_tg
 * may be NULL to run one network. */
int t2o_agent_unroll_fwd(const t2o_layout* L, const float* pack_on, const float* pack_tg,
                         const float* obs, int64_t obs_sb, int64_t obs_st,
                         const float* h0_on, const float* h0_tg,
                         float* q_on, float* h_on, float* q_tg, float* h_tg,
                         int B, int T, int A, void* stream);

/* Agent BPTT over steps T-1..0 of one network.  h_seq = forward h output
 * [b][h_ts][a][E] (h_ts >= T), h0 as in the forward (NULL = zeros).  External
 * grads of the T steps: gq[b][t][a][NA] (may be NULL) plus, if gchosen != NULL,
 * gchosen[b][t][a] routed to q[action] (actions int64 [b][t][a] with element
 * strides act_sb, act_st, a-stride 1); gh[b][t][a][E] (may be NULL).
 * Outputs: gslabs[nslab][grad_total] per-workgroup partial gradients (compact
 * layout, overwritten; *nslab = number written, at most max_slabs =
 * t2o_agent_bwd_max_slabs(B, A)); gh0[b][a][E] = dL/dh0 (may be NULL). */
int t2o_agent_unroll_bwd(const t2o_layout* L, const float* pack,
                         const float* obs, int64_t obs_sb, int64_t obs_st,
                         const float* h0, const float* h_seq, int h_ts,
                         const float* gq, const float* gchosen, const int64_t* actions,
                         int64_t act_sb, int64_t act_st, const float* gh,
                         float* gslabs, int max_slabs, int* nslab, float* gh0,
                         int B, int T, int A, void* stream);
int t2o_agent_bwd_max_slabs(int B, int A);

/* Sum nslab partial gradient slabs [nslab][n] into out[n] (out = sum, overwritten). */
int t2o_reduce_slabs(const float* slabs, int nslab, int64_t n, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* T2OMCA_H */
