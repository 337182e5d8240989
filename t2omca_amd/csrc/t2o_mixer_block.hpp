// t2o_mixer_block.hpp — one transformer block of the mixer for a 16-query tile.
//
// Reference: n_transf_mixer.py:55-91 -> transformer.py:40-140.  The mixer's
// tokens for one (episode, t) are X0 = [We·s_j + b_e (A state entities),
// agent hidden states (A), hyper-weight tokens (3)]; only the last A+3 rows
// are read out (w1, b1, w2, b2 — n_transf_mixer.py:75-85), and keys never
// change across blocks (transformer.py:140), so only those A+3 query rows are
// propagated.  A wave owns ONE episode: queries sit on the MFMA N axis (lanes),
// the key block X0 [keys x E] is built in wave-private LDS once per step and
// held in registers as MFMA fragments (KeyFrags), and per head
//   Sᵀ = X0 · u_h        (u_h = M_h x, scores for all keys of all queries)
//   Zᵀ = X0ᵀ · softmax(S)ᵀ
// are two MFMA products whose outputs are already in the T-layout the next
// step consumes (keys on the register axis for S, features for Z).
#pragma once
#include <type_traits>

#include "t2o_block.hpp"

namespace t2o {

template <int E, int H, int KT, int FF>
struct MixerCache {
  static constexpr int ET = E / 16, HET = H * ET;
  PostCache<E, H, FF> post;
  f4 u[HET];
  f4 p[H][KT];
};

// The key block X0 of one (episode, step) as MFMA A-operand fragments, read
// from the wave's LDS copy once per step and reused by every head of every
// block (and by the backward's products):
//   dot[kt][ft]  = X0[key 16kt + c][features 16ft + 4g .. +3]   (Sᵀ = X0 · v)
//   comb[kt][ft] = X0[keys 16kt + 4g .. +3][feature 16ft + c]    (Zᵀ = X0ᵀ · w)
// fp32 holds them as f32.  bf16 pairs the contraction's 16-wide K tiles into
// 16x16x32 operands — dot8[kt][p] = (dot[kt][2p], dot[kt][2p+1]) over feature
// tiles, comb8[p][ft] = (comb[2p][ft], comb[2p+1][ft]) over key tiles (an odd
// feature-tile count's last tile alone in dot1; an odd key-tile count: every
// comb tile alone in comb1) — so each product takes half the MFMAs
// and its B operand (u_h, gz_h; the probabilities) converts 8-wide, i.e. packed
// (to_bf4: the 4-wide conversions of round 4 cost six VALU per tile).
// KM 1 (fp32 only): the fragments are read from LDS at each product instead of held
// in registers — dot from the key block X0 itself, comb from a transposed copy X0T
// ([feature][key], row stride 16 KT + 4) the kernel writes once per step.  The
// one-wave BPTT kernels of the 32- / 64-agent capacity classes (KT >= 5) use it: their
// 16·KT fragment registers beside KT·8 key-grad accumulators spilled 1-6 KB a lane.
template <int KT, typename WT>
constexpr int key_mode() { return sizeof(WT) == 4 && KT >= 5 ? 1 : 0; }

template <int E, int KT, bool BF, int KM = 0>
struct KeyFrags {
  static_assert(KM == 0 || !BF, "LDS-read key fragments: fp32 only");
  static constexpr bool IN_LDS = KM == 1;
  static constexpr int LDXK = E + 4, LDT = 16 * KT + 4;  // X0 (MixDims::LDX) / X0T row strides
  static constexpr int X0T_FLOATS = IN_LDS ? E * LDT : 0;
  // An odd key-tile count (16 / 20 / 64 AGVs) keeps every comb tile unpaired.  Paired
  // tiles plus a lone tail chain a 16x16x16 MFMA onto a 16x16x32 result in place, and
  // hipcc (ROCm 7.2) issues that pair with 0-4 wait states: on gfx950 the 16x16x16
  // then reads a stale accumulator (t2o_probe_xdl_hazards: 3662 of 4096 waves wrong
  // at 0 states, 3775 at 4; the same opcode back to back is exact).  That was round
  // 5's run-to-run nondeterminism of the odd-pairing build (profiles/r5_bis/); with
  // the tail padded or summed on its own it was exact and reproducible, and no faster
  // (configs[0]-shape 3.640 / 3.663 vs 3.646 ms, 64 AGVs 40.41 / 40.45 vs 39.96 ms,
  // profiles/r6_check/), so odd counts stay unpaired.
  static constexpr int ET = E / 16, EP = ET / 2;
  static constexpr int KP = (KT & 1) ? 0 : KT / 2;
  static constexpr bool EO = EP * 2 != ET, KO = KP * 2 != KT;
  // EU / KU unpaired feature / key tiles (the last ones: 2 EP .. ET-1, 2 KP .. KT-1)
  static constexpr int N_EP = EP > 0 ? EP : 1, N_KP = KP > 0 ? KP : 1, EU = ET - 2 * EP, KU = KT - 2 * KP;
  // fp32
  f4 dot[BF || IN_LDS ? 1 : KT][BF || IN_LDS ? 1 : ET], comb[BF || IN_LDS ? 1 : KT][BF || IN_LDS ? 1 : ET];
  const float* x0 = nullptr;   // IN_LDS: the key block and its transposed copy
  const float* x0t = nullptr;
  // bf16
  bf8 dot8[BF ? KT : 1][N_EP], comb8[BF ? N_KP : 1][ET];
  bf4 dot1[BF && EO ? KT : 1][EO ? EU : 1], comb1[BF && KO ? KU : 1][ET];
  // IN_LDS: bind the block (X0T written by write_transposed, wave-synchronised)
  T2O_DEV void bind(const float* X0, const float* X0T) {
    x0 = X0;
    x0t = X0T;
  }
  // X0T[f][k] = X0[k][f] for the KT·16 key rows (call after X0 is complete, then wave_sync)
  static T2O_DEV void write_transposed(const float* X0, float* X0T) {
    for (int i = threadIdx.x & 63; i < 16 * KT * E; i += 64) X0T[(i % E) * LDT + i / E] = X0[(i / E) * LDXK + i % E];
  }
  T2O_DEV f4 dotf(int kt, int ft) const {
    if constexpr (IN_LDS) return ld4(x0 + (16 * kt + lane_c()) * LDXK + 16 * ft + 4 * lane_g());
    else return dot[kt][ft];
  }
  T2O_DEV f4 combf(int kt, int ft) const {
    if constexpr (IN_LDS) return ld4(x0t + (16 * ft + lane_c()) * LDT + 16 * kt + 4 * lane_g());
    else return comb[kt][ft];
  }
  template <int LDX>
  T2O_DEV void load(const float* __restrict__ X0) {
    static_assert(!IN_LDS, "LDS-read fragments: bind()");
    const int c = lane_c(), g = lane_g();
    auto arow = [&](int kt, int ft) { return ld4(X0 + (16 * kt + c) * LDX + 16 * ft + 4 * g); };
    auto bcol = [&](int kt, int ft) {
      f4 b;
#pragma unroll
      for (int s = 0; s < 4; ++s) b[s] = X0[(16 * kt + 4 * g + s) * LDX + 16 * ft + c];
      return b;
    };
    if constexpr (BF) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
        for (int p = 0; p < EP; ++p) dot8[kt][p] = cvt8(arow(kt, 2 * p), arow(kt, 2 * p + 1));
        if constexpr (EO)
#pragma unroll
          for (int u = 0; u < EU; ++u) dot1[kt][u] = to_bf4(arow(kt, 2 * EP + u));
      }
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) {
#pragma unroll
        for (int p = 0; p < KP; ++p) comb8[p][ft] = cvt8(bcol(2 * p, ft), bcol(2 * p + 1, ft));
        if constexpr (KO)
#pragma unroll
          for (int u = 0; u < KU; ++u) comb1[u][ft] = to_bf4(bcol(2 * KP + u, ft));
      }
    } else {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ft = 0; ft < ET; ++ft) {
          dot[kt][ft] = arow(kt, ft);
          comb[kt][ft] = bcol(kt, ft);
        }
    }
  }
};

// The step's key fragments: into registers (KM 0), or X0T written and the LDS copy
// bound (KM 1).  X0 must be complete and wave-synchronised; X0T's previous readers done.
template <int LDX, int E, int KT, bool BF, int KM>
T2O_DEV void load_keys(KeyFrags<E, KT, BF, KM>& K, const float* X0, float* X0T) {
  if constexpr (KM == 1) {
    KeyFrags<E, KT, BF, KM>::write_transposed(X0, X0T);
    wave_sync();
    K.bind(X0, X0T);
  } else {
    (void)X0T;
    K.template load<LDX>(X0);
  }
}

T2O_DEV f4 mfma_b8(bf8 a, bf8 b, f4 acc) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0); }

// Sᵀ-style product: out[kt] (keys 16kt+4g+r, query c) = Σ_f X0[key][f] v[f]
template <int E, int KT, bool BF, int KM>
T2O_DEV void keys_dot(const KeyFrags<E, KT, BF, KM>& K, const f4* v, f4* out) {
  using KF = KeyFrags<E, KT, BF, KM>;
  constexpr int ET = E / 16;
  if constexpr (BF) {
    bf8 vb[KF::N_EP];
    bf4 vt[KF::EO ? KF::EU : 1];
#pragma unroll
    for (int p = 0; p < KF::EP; ++p) vb[p] = cvt8(v[2 * p], v[2 * p + 1]);
    if constexpr (KF::EO)
#pragma unroll
      for (int u = 0; u < KF::EU; ++u) vt[u] = to_bf4(v[2 * KF::EP + u]);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      f4 acc = zero4();
#pragma unroll
      for (int p = 0; p < KF::EP; ++p) acc = mfma_b8(K.dot8[kt][p], vb[p], acc);
      if constexpr (KF::EO)
#pragma unroll
        for (int u = 0; u < KF::EU; ++u) acc = chain_tail_b16<(KF::EP > 0)>(K.dot1[kt][u], vt[u], acc);
      out[kt] = acc;
    }
  } else {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      f4 acc = zero4();
#pragma unroll
      for (int ft = 0; ft < ET; ++ft) {
        const f4 d = K.dotf(kt, ft);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(d[s], v[ft][s], acc);
      }
      out[kt] = acc;
    }
  }
}

// Zᵀ-style product: out[ft] (features 16ft+4g+r, query c) = Σ_key X0[key][f] w[key]
template <int E, int KT, bool BF, int KM>
T2O_DEV void keys_combine(const KeyFrags<E, KT, BF, KM>& K, const f4* w, f4* out) {
  using KF = KeyFrags<E, KT, BF, KM>;
  constexpr int ET = E / 16;
  if constexpr (BF) {
    bf8 wb[KF::N_KP];
    bf4 wt[KF::KO ? KF::KU : 1];
#pragma unroll
    for (int p = 0; p < KF::KP; ++p) wb[p] = cvt8(w[2 * p], w[2 * p + 1]);
    if constexpr (KF::KO)
#pragma unroll
      for (int u = 0; u < KF::KU; ++u) wt[u] = to_bf4(w[2 * KF::KP + u]);
#pragma unroll
    for (int ft = 0; ft < ET; ++ft) {
      f4 acc = zero4();
#pragma unroll
      for (int p = 0; p < KF::KP; ++p) acc = mfma_b8(K.comb8[p][ft], wb[p], acc);
      static_assert(!(KF::KO && KF::KP > 0), "a 16x16x16 chained onto a 16x16x32 accumulator (see KeyFrags)");
      if constexpr (KF::KO)
#pragma unroll
        for (int u = 0; u < KF::KU; ++u) acc = mfma_b16(K.comb1[u][ft], wt[u], acc);
      out[ft] = acc;
    }
  } else {
#pragma unroll
    for (int ft = 0; ft < ET; ++ft) {
      f4 acc = zero4();
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const f4 b = K.combf(kt, ft);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(b[s], w[kt][s], acc);
      }
      out[ft] = acc;
    }
  }
}

// scores of keys >= Lk (padding) to -inf.  bf16: per element and branch-free (a
// wave-uniform "does this tile reach Lk" test per tile measured slower where Lk is a
// run-time value: 32 AGVs mixer_bwd 7.49 vs 6.56 ms, profiles/r5_km/).  fp32 keeps the
// per-tile test: built branch-free, the capacity-64 split BPTT returned wrong
// gradients although both forms mask the same elements; the cause is not named
// (not an MFMA hand-off, not LDS ordering, not the frame size)
template <int KT, bool TILE_TEST>
T2O_DEV void key_mask(f4* s, int Lk, int g) {
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
    if (!TILE_TEST || 16 * kt + 16 > Lk) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (16 * kt + 4 * g + r >= Lk) s[kt][r] = -INFINITY;
    }
}

// HOIST: matvec's swizzle hoisting (t2o_common.hpp), true from the forward kernel
template <int E, int H, int KT, int FF, bool CACHE, typename WT, bool HOIST = T2O_SWZ_HOIST, int KM = 0>
T2O_DEV void mixer_block_fwd(const Wts<WT>& P, const t2o_layout& L, int d,
                             const KeyFrags<E, KT, sizeof(WT) == 2, KM>& K, int Lk, f4* x,
                             MixerCache<E, H, KT, FF>* cache) {
  constexpr int ET = E / 16, HET = H * ET;
  constexpr bool BF = sizeof(WT) == 2;
  const int g = lane_g();
  f4 u[HET];
  matvec<HET, ET, HOIST>(P.w + L.M[d], E, x, u, P.vol);
  f4 z[HET];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    f4 s[KT];
    keys_dot(K, &u[hh * ET], s);
    key_mask<KT, !BF>(s, Lk, g);
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) m = fmaxf(m, s[kt][r]);
    m = allmax4(m);
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[kt][r] = exp_fast(s[kt][r] - m);
        l += s[kt][r];
      }
    const float il = rcp_fast(allsum4(l));
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) s[kt] *= il;
    keys_combine(K, s, &z[hh * ET]);
    if constexpr (CACHE) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) cache->p[hh][kt] = s[kt];
    }
  }
  if constexpr (CACHE) {
#pragma unroll
    for (int t = 0; t < HET; ++t) cache->u[t] = u[t];
  }
  post_fwd<E, H, FF, CACHE, WT, HOIST>(P, L, d, z, x, CACHE ? &cache->post : nullptr);
}

// Backward of block d for one query tile.  gx: in = grad wrt block output,
// out = grad wrt block input.  gX0 — MFMA accumulator registers, tile [kt][ft]
// holds gX0[key 16kt+4g+r][feature 16ft+c] — accumulates the grad wrt the key
// tokens (a contraction over queries = rows, via the staging transposes).
// Big-matrix operand pairs go to the query row's tape record (null = padding).
template <int E, int H, int KT, int FF, typename WT, int KM = 0>
T2O_DEV void mixer_block_bwd(const Wts<WT>& P, const t2o_layout& L, const t2o_layout& G,
                             float* __restrict__ gs, WT* __restrict__ rec, float* __restrict__ stage, int d,
                             const KeyFrags<E, KT, sizeof(WT) == 2, KM>& K, f4 (&gX0)[KT][E / 16],
                             const MixerCache<E, H, KT, FF>& c, f4* gx, f4* ln2) {
  constexpr int ET = E / 16, HET = H * ET;
  constexpr bool BF = sizeof(WT) == 2;
  f4 gz[HET], gres[ET];
  post_bwd<E, H, FF>(P, L, G, gs, rec, d, c.post, gx, gz, gres, ln2);
  f4 gu[HET];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    f4 gp[KT];
    keys_dot(K, &gz[hh * ET], gp);
    float dot = 0.f;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dot += c.p[hh][kt][r] * gp[kt][r];
    dot = allsum4(dot);
    f4 gsc[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) gsc[kt] = c.p[hh][kt] * (gp[kt] - dot);
    keys_combine(K, gsc, &gu[hh * ET]);
    dw_accumulate_regs<KT, ET, BF>(gX0, c.p[hh], &gz[hh * ET], stage);
    dw_accumulate_regs<KT, ET, BF>(gX0, gsc, &c.u[hh * ET], stage);
  }
  if (rec) {
    rec_store<TapeRec<E, H, FF>::SIZE, HET>(rec, TapeRec<E, H, FF>::GU, gu);
    rec_store<TapeRec<E, H, FF>::SIZE, ET>(rec, TapeRec<E, H, FF>::X, c.post.x);
  }
  f4 gxp[ET];
  matvec_tr<ET, HET>(P, L.M[d], E, L.MT[d], H * E, gu, gxp);
#pragma unroll
  for (int t = 0; t < ET; ++t) gx[t] = gxp[t] + gres[t];
}

// Lean cache (PostCacheLean) versions for the two-wave pipelined backward:
// the forward recompute writes the record's X, Z, Y fields itself.  With many
// key tiles (KT > 4: 64 agents) the attention probabilities are not cached but
// recomputed from u in the backward (KT MFMAs per head against 12·KT registers
// per head held across the post-attention backward).
template <int E, int H, int KT, int FF>
struct MixerCacheLean {
  static constexpr int ET = E / 16, HET = H * ET;
  static constexpr bool PC = KT <= 4;
  PostCacheLean<E, H, FF> post;
  f4 u[HET];
  f4 p[PC ? H : 1][PC ? KT : 1];
};

// softmax over the Lk valid keys of one head's scores: s[kt] (keys 16kt+4g+r, query c)
template <int E, int KT, bool BF, int KM>
T2O_DEV void attn_probs(const KeyFrags<E, KT, BF, KM>& K, const f4* u, int Lk, f4* s) {
  const int g = lane_g();
  keys_dot(K, u, s);
  key_mask<KT, !BF>(s, Lk, g);
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) m = fmaxf(m, s[kt][r]);
  m = allmax4(m);
  float l = 0.f;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[kt][r] = exp_fast(s[kt][r] - m);
      l += s[kt][r];
    }
  const float il = rcp_fast(allsum4(l));
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) s[kt] *= il;
}

template <int E, int H, int KT, int FF, typename WT, int CP, int KM = 0>
T2O_DEV void mixer_block_fwd_lean(const Wts<WT>& P, const t2o_layout& L, int d,
                                  const KeyFrags<E, KT, sizeof(WT) == 2, KM>& K, int Lk, f4* x,
                                  MixerCacheLean<E, H, KT, FF>& cache, const MaskedRec<WT, CP>& rec) {
  constexpr int ET = E / 16, HET = H * ET;
  constexpr bool BF = sizeof(WT) == 2;
  matvec<HET, ET>(P.w + L.M[d], E, x, cache.u, P.vol);
  f4 z[HET];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    f4 s[KT];
    attn_probs(K, &cache.u[hh * ET], Lk, s);
    if constexpr (MixerCacheLean<E, H, KT, FF>::PC) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) cache.p[hh][kt] = s[kt];
    }
    keys_combine(K, s, &z[hh * ET]);
  }
  post_fwd_lean<E, H, FF>(P, L, d, z, x, &cache.post, rec);
}

template <int E, int H, int KT, int FF, typename WT, int CP, int KM = 0>
T2O_DEV void mixer_block_bwd_lean(const Wts<WT>& P, const t2o_layout& L, float* __restrict__ gs,
                                  const MaskedRec<WT, CP>& rec, float* __restrict__ stage, int d,
                                  const KeyFrags<E, KT, sizeof(WT) == 2, KM>& K, int Lk, f4 (&gX0)[KT][E / 16],
                                  const MixerCacheLean<E, H, KT, FF>& c, f4* gx, f4* ln2) {
  constexpr int ET = E / 16, HET = H * ET;
  constexpr bool BF = sizeof(WT) == 2;
  f4 gz[HET], gres[ET];
  post_bwd_lean<E, H, FF>(P, L, gs, rec, d, c.post, gx, gz, gres, ln2);
  f4 gu[HET];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    f4 p[KT];
    if constexpr (MixerCacheLean<E, H, KT, FF>::PC) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) p[kt] = c.p[hh][kt];
    } else {
      attn_probs(K, &c.u[hh * ET], Lk, p);
    }
    f4 gp[KT];
    keys_dot(K, &gz[hh * ET], gp);
    float dot = 0.f;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dot += p[kt][r] * gp[kt][r];
    dot = allsum4(dot);
    f4 gsc[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) gsc[kt] = p[kt] * (gp[kt] - dot);
    keys_combine(K, gsc, &gu[hh * ET]);
    dw_accumulate_regs<KT, ET, BF>(gX0, p, &gz[hh * ET], stage);
    dw_accumulate_regs<KT, ET, BF>(gX0, gsc, &c.u[hh * ET], stage);
  }
  rec.template store<HET>(TapeRec<E, H, FF>::GU, gu);
  f4 gxp[ET];
  matvec_tr<ET, HET>(P, L.M[d], E, L.MT[d], H * E, gu, gxp);
#pragma unroll
  for (int t = 0; t < ET; ++t) gx[t] = gxp[t] + gres[t];
}

}  // namespace t2o
