// t2o_dispatch.hpp — runtime (E, H, D, n_ent, FF) -> compile-time kernel instance.
//
// Two kinds of MFMA instance:
//   exact    the entity count is a compile-time constant: the reference
//            defaults of BASELINE configs 0-4 (emb 32, 3 heads, depth 2,
//            ff_hidden_mult 4 at 8, 16 or 64 AGVs) plus the fixture shapes
//            (3 AGVs; emb 16 / 2 heads / depth 1).
//   runtime  the same network at ANY entity count 1..64 (environment_multi_mec.py:9-11
//            takes any agv_num): the kernel is compiled for a capacity class —
//            register arrays, key / query tile counts sized for it — and reads
//            the real count from its arguments; padding entities / keys / query
//            rows are masked (softmax -inf, zero operands, no stores).
// Inside a kernel `NE_` is the exact count or the capacity and `RT_` says which.
// Every other shape is laid out generic (t2o_layout_init) and runs the
// runtime-shaped scalar kernels of t2o_generic.hip.
#pragma once

// the default network of every BASELINE config (emb 32, heads 3, depth 2, FF 128)
inline bool t2o_default_net(int E, int H, int D, int FF) { return E == 32 && H == 3 && D == 2 && FF == 128; }

inline bool t2o_exact_shape(int E, int H, int D, int NE, int FF) {
  return (E == 16 && H == 2 && D == 1 && NE == 3 && FF == 64) ||
         (t2o_default_net(E, H, D, FF) && (NE == 3 || NE == 8 || NE == 16 || NE == 64));
}

// the list t2o_layout_init consults (shapes outside it get generic = 1)
inline bool t2o_tuned_shape(int E, int H, int D, int NE, int FF) {
  return t2o_exact_shape(E, H, D, NE, FF) || (t2o_default_net(E, H, D, FF) && NE >= 1 && NE <= 64);
}

// Capacity classes of the runtime instances.
//   agent: 8 / 16 entities in registers, 64 streamed in 8-entity chunks
//   mixer: 8 and 13 agents fit one 16-row query tile (A + 3 <= 16: the
//          two-wave pipelined BPTT), 16 / 32 / 64 the multi-tile kernels
inline int t2o_agent_cap(int ne) { return ne <= 8 ? 8 : ne <= 16 ? 16 : 64; }
inline int t2o_mixer_cap(int a) { return a <= 8 ? 8 : a <= 13 ? 13 : a <= 16 ? 16 : a <= 32 ? 32 : 64; }

#define T2O_CASE_X(E, H, D, NE, FF, RT, STMT)                               \
  {                                                                          \
    constexpr int E_ = E, H_ = H, D_ = D, NE_ = NE, FF_ = FF;                \
    constexpr bool RT_ = (RT) != 0;                                          \
    constexpr int RTM_ = RT;                                                 \
    (void)E_; (void)H_; (void)D_; (void)NE_; (void)FF_; (void)RT_; (void)RTM_; \
    STMT;                                                                    \
  }

#define T2O_DISPATCH_EXACT(STMT)                                                        \
  if (e_ == 16 && h_ == 2 && d_ == 1 && ne_ == 3 && ff_ == 64) T2O_CASE_X(16, 2, 1, 3, 64, false, STMT)  \
  else if (t2o_default_net(e_, h_, d_, ff_) && ne_ == 3) T2O_CASE_X(32, 3, 2, 3, 128, false, STMT)        \
  else if (t2o_default_net(e_, h_, d_, ff_) && ne_ == 8) T2O_CASE_X(32, 3, 2, 8, 128, false, STMT)        \
  else if (t2o_default_net(e_, h_, d_, ff_) && ne_ == 16) T2O_CASE_X(32, 3, 2, 16, 128, false, STMT)      \
  else if (t2o_default_net(e_, h_, d_, ff_) && ne_ == 64) T2O_CASE_X(32, 3, 2, 64, 128, false, STMT)

// agent kernels: exact instance, else the runtime instance of the entity count's class
#define T2O_DISPATCH_AGENT(EV, HV, DV, NEV, FFV, STMT)                                          \
  do {                                                                                          \
    const int e_ = (EV), h_ = (HV), d_ = (DV), ne_ = (NEV), ff_ = (FFV);                        \
    T2O_DISPATCH_EXACT(STMT)                                                                    \
    else if (t2o_default_net(e_, h_, d_, ff_) && ne_ >= 1 && ne_ <= 64) {                       \
      const int cap_ = t2o_agent_cap(ne_);                                                      \
      if (cap_ == 8) T2O_CASE_X(32, 3, 2, 8, 128, true, STMT)                                   \
      else if (cap_ == 16) T2O_CASE_X(32, 3, 2, 16, 128, true, STMT)                            \
      else T2O_CASE_X(32, 3, 2, 64, 128, true, STMT)                                            \
    }                                                                                           \
  } while (0)

// mixer kernels: exact instance (abs head), else the runtime instance of the agent
// count's class (which also computes the other qmix_pos_funcs).  RTM_ (the
// mixer's instance mode): 0 exact counts + abs head, 1 runtime counts + runtime
// head, 2 exact counts + runtime head — the headline's 8 AGVs with a softplus /
// quadratic / identity head (the runtime instance's register file holds the
// counts too and spilled: 1.05 vs 0.57 ms mixer BPTT, profiles/r3_f5/softplus.json)
#define T2O_DISPATCH_MIXER(EV, HV, DV, NEV, FFV, ABS, STMT)                                     \
  do {                                                                                          \
    const int e_ = (EV), h_ = (HV), d_ = (DV), ne_ = (NEV), ff_ = (FFV);                        \
    if ((ABS) && t2o_exact_shape(e_, h_, d_, ne_, ff_)) {                                       \
      T2O_DISPATCH_EXACT(STMT)                                                                  \
    } else if (!(ABS) && t2o_default_net(e_, h_, d_, ff_) && ne_ == 8) {                        \
      T2O_CASE_X(32, 3, 2, 8, 128, 2, STMT)                                                     \
    } else if (t2o_default_net(e_, h_, d_, ff_) && ne_ >= 1 && ne_ <= 64) {                     \
      const int cap_ = t2o_mixer_cap(ne_);                                                      \
      if (cap_ == 8) T2O_CASE_X(32, 3, 2, 8, 128, true, STMT)                                   \
      else if (cap_ == 13) T2O_CASE_X(32, 3, 2, 13, 128, true, STMT)                            \
      else if (cap_ == 16) T2O_CASE_X(32, 3, 2, 16, 128, true, STMT)                            \
      else if (cap_ == 32) T2O_CASE_X(32, 3, 2, 32, 128, true, STMT)                            \
      else T2O_CASE_X(32, 3, 2, 64, 128, true, STMT)                                            \
    }                                                                                           \
  } while (0)

// entity-count-independent kernels (the tape contraction): one instance per network
#define T2O_DISPATCH_NET(EV, HV, DV, FFV, STMT)                                                 \
  do {                                                                                          \
    const int e_ = (EV), h_ = (HV), d_ = (DV), ff_ = (FFV);                                     \
    if (e_ == 16 && h_ == 2 && d_ == 1 && ff_ == 64) T2O_CASE_X(16, 2, 1, 0, 64, false, STMT)   \
    else if (t2o_default_net(e_, h_, d_, ff_)) T2O_CASE_X(32, 3, 2, 0, 128, false, STMT)        \
  } while (0)
