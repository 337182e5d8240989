// t2o_generic.hpp — entry points of the runtime-shaped kernels (t2o_generic.hip).
// Same arguments as the C-ABI functions of include/t2omca.h they serve; the
// C-ABI functions forward here when the layout says generic = 1.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/t2omca.h"

namespace t2o {

int gen_agent_unroll_fwd(const t2o_layout* L, const float* pack_on, const float* pack_tg, const float* obs,
                         int64_t obs_sb, int64_t obs_st, const float* h0_on, const float* h0_tg, float* q_on,
                         float* h_on, float* hmid_on, float* q_tg, float* h_tg, float* hmid_tg, int B, int T, int A,
                         hipStream_t stream);

int gen_agent_unroll_bwd(const t2o_layout* L, const float* pack, const float* obs, int64_t obs_sb, int64_t obs_st,
                         const float* h0, const float* h_seq, const float* hmid, int h_ts, const float* gq,
                         const float* gchosen, const int64_t* actions, int64_t act_sb, int64_t act_st,
                         const float* gh, float* gslabs, int max_slabs, int* nslab, void* tape, float* gh0, int B,
                         int T, int A, hipStream_t stream);

int gen_mixer_unroll_fwd(const t2o_layout* L, const float* pack_on, const float* pack_tg, const float* states,
                         int64_t st_sb, int64_t st_st, const float* hid_on, const float* hid_tg, int64_t hid_sb,
                         int64_t hid_st, const float* hw0_on, const float* hw0_tg, int qmode_on, int qmode_tg,
                         const float* qv_on, const float* qv_tg, const float* q_on, const float* q_tg, int q_ts,
                         int n_actions, const int64_t* actions, int64_t act_sb, int64_t act_st,
                         const int32_t* avail, int64_t av_sb, int64_t av_st, float* y_on, float* hw_on,
                         float* qvo_on, float* xout_on, float* xmid_on, float* y_tg, float* hw_tg, float* qvo_tg,
                         float* xout_tg, float* xmid_tg, int B, int T_on, int T_tg, hipStream_t stream);

int gen_mixer_unroll_bwd(const t2o_layout* L, const float* pack, const float* states, int64_t st_sb, int64_t st_st,
                         const float* hid, int64_t hid_sb, int64_t hid_st, const float* hw0, const float* qv,
                         const float* hw, const float* xout, const float* xmid, const float* gy,
                         const float* ghw_ext, float* gqv, float* ghid, float* ghw0, float* gslabs, int max_slabs,
                         int* nslab, void* tape, int B, int T, hipStream_t stream);

int64_t gen_tape_floats(const t2o_layout* L, int64_t tiles);

int gen_tape_contract(const t2o_layout* L, const void* tape, int64_t tiles, float* gslabs, int nslab,
                      hipStream_t stream);

}  // namespace t2o
