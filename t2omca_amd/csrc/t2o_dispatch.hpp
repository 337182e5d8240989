// t2o_dispatch.hpp — runtime (E, H, D, n_ent, FF) -> compile-time kernel instance.
//
// Instantiated shapes: the reference defaults used by BASELINE configs 1-4
// (emb 32, 3 heads, depth 2, ff_hidden_mult 4, 8, 16 or 64 AGVs) plus the
// small shapes of the golden fixtures.  (64 AGVs runs the generic code with
// register spills: correct, not tuned — DESIGN.md §9.)  Anything else returns T2O_EUNSUPPORTED
// (the Python side raises; there is no fallback path).
#pragma once

#define T2O_CASE(E, H, D, NE, FF, STMT)                                   \
  if (e_ == E && h_ == H && d_ == D && ne_ == NE && ff_ == FF) {           \
    constexpr int E_ = E, H_ = H, D_ = D, NE_ = NE, FF_ = FF;              \
    (void)E_; (void)H_; (void)D_; (void)NE_; (void)FF_;                    \
    STMT;                                                                  \
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
