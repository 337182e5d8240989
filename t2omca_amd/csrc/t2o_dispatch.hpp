// t2o_dispatch.hpp — runtime (E, H, D, n_ent, FF) -> compile-time kernel instance.
//
// Instantiated shapes: the reference defaults used by BASELINE configs 1-4
// (emb 32, 3 heads, depth 2, ff_hidden_mult 4, 8, 16 or 64 AGVs) plus the
// small shapes of the golden fixtures.  Every other shape is laid out generic
// (t2o_layout_init) and runs the runtime-shaped kernels of t2o_generic.hip.
#pragma once

#define T2O_CASE(E, H, D, NE, FF, STMT)                                   \
  if (e_ == E && h_ == H && d_ == D && ne_ == NE && ff_ == FF) {           \
    constexpr int E_ = E, H_ = H, D_ = D, NE_ = NE, FF_ = FF;              \
    (void)E_; (void)H_; (void)D_; (void)NE_; (void)FF_;                    \
    STMT;                                                                  \
  }

// the same list, for t2o_layout_init (shapes outside it get generic = 1)
inline bool t2o_tuned_shape(int E, int H, int D, int NE, int FF) {
  return (E == 16 && H == 2 && D == 1 && NE == 3 && FF == 64) ||
         (E == 32 && H == 3 && D == 2 && FF == 128 && (NE == 3 || NE == 8 || NE == 16 || NE == 64));
}

#define T2O_DISPATCH(EV, HV, DV, NEV, FFV, STMT)                          \
  do {                                                                     \
    const int e_ = (EV), h_ = (HV), d_ = (DV), ne_ = (NEV), ff_ = (FFV);   \
    T2O_CASE(16, 2, 1, 3, 64, STMT)                                        \
    else T2O_CASE(32, 3, 2, 3, 128, STMT)                                  \
    else T2O_CASE(32, 3, 2, 8, 128, STMT)                                  \
    else T2O_CASE(32, 3, 2, 16, 128, STMT)                                 \
    else T2O_CASE(32, 3, 2, 64, 128, STMT)                                 \
  } while (0)
