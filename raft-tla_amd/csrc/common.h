// raftmc — common device/host helpers (gfx950 product code).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define RMC_HD __host__ __device__ __forceinline__
#define RMC_DEV __device__ __forceinline__
#else
#define RMC_HD inline
#define RMC_DEV inline
#endif

namespace rmc {

typedef uint32_t u32;
typedef uint64_t u64;
typedef int32_t i32;
typedef int64_t i64;

// number of bits needed to hold every value in 0..x
constexpr int bits_for(long long x) { int b = 1; while ((1LL << b) <= x) ++b; return b; }
constexpr long long ipow(long long b, int e) { long long r = 1; for (int k = 0; k < e; ++k) r *= b; return r; }
constexpr long long log_universe(long long e, int ml) { long long u = 0, pw = 1; for (int k = 0; k <= ml; ++k) { u += pw; pw *= e; } return u; }
constexpr u64 lomask(int w) { return w >= 64 ? ~0ull : ((1ull << w) - 1ull); }

// Fixed-width sub-field k of a packed scalar word (runtime k -> variable shift, stays in registers).
template <int W, class T> RMC_HD T fget(T x, int k) { return (T)((x >> (k * W)) & (T)lomask(W)); }
template <int W, class T> RMC_HD void fset(T& x, int k, T v) {
  const T m = (T)lomask(W) << (k * W);
  x = (T)((x & ~m) | (((T)v << (k * W)) & m));
}
template <int W, class T> RMC_HD T fsplat(T v, int n) { T r = 0; for (int k = 0; k < n; ++k) r |= (T)v << (k * W); return r; }

// Runtime-indexed read/write of a small register array without scratch.  The
// array is a value type and `sel` takes it BY VALUE: inside sel the copy is
// promoted to SSA values first, so the select chain stays a chain of
// v_cndmask (a reference parameter lets instcombine fold it back into a
// dynamically indexed load, which pins the whole state struct in scratch).
template <class T, int N> struct Arr { T v[N]; };
template <class T, int N> RMC_HD T sel(Arr<T, N> a, int i) {
  T r = a.v[0];
#pragma unroll
  for (int k = 1; k < N; ++k) r = (i == k) ? a.v[k] : r;
  return r;
}
template <class T, int N> RMC_HD void put(Arr<T, N>& a, int i, T x) {
#pragma unroll
  for (int k = 0; k < N; ++k) a.v[k] = (i == k) ? x : a.v[k];
}

RMC_HD int popc32(u32 x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popc(x);
#else
  return __builtin_popcount(x);
#endif
}

// ---------------------------------------------------------------------------
// FP64 of raftmc: a sum of xxHash64-style per-word mixes over the packed state words (two
// 64-bit multiplies per 8 bytes, keyed by the word's position and the seed).  The seed is fixed
// per run and recorded in the summary.  0 is the empty-slot marker of the
// seen-set, so a fingerprint of 0 is remapped to 1 (documented bias 2^-64).
// ---------------------------------------------------------------------------
constexpr u64 P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
              P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
RMC_HD u64 rotl64(u64 x, int r) { return (x << r) | (x >> (64 - r)); }
RMC_HD u64 fmix64(u64 h) { h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32; return h; }
// the fingerprint from the sum of the per-word terms: the sum itself.  (Rounds 1-5 followed it with
// xxh64's avalanche, fmix64(acc ^ seed ^ NW * P4): a bijection, so it changed no collision -- two states
// collide iff their sums do -- only the bits the seen-set indexes by, and a sum of fmix64 outputs is as
// uniform in every bit.  Dropping it saves one fmix64 per successor: orig_generate 11.67 -> 11.14 ms
// per C2 run, round 6, profiles/r06_generate_ab.txt.)
template <int NW32>
RMC_HD u64 fp_final(u64 acc, u64 seed) {
  (void)seed;
  return acc ? acc : 1ull;
}
template <int NW32>
RMC_HD u64 fp64(const u32 (&w)[NW32], u64 seed) {
  // per 64-bit word a bijective mix keyed by its position, summed: equal fingerprints need equal
  // words or a 2^-64 coincidence of mixes
  u64 acc = 0;
#pragma unroll
  for (int k = 0; k < NW32; k += 2) {
    const u64 v = (u64)w[k] | (k + 1 < NW32 ? (u64)w[k + 1] << 32 : 0ull);
    acc += fmix64(v ^ (seed + (u64)(k / 2 + 1) * P1));
  }
  return fp_final<NW32>(acc, seed);
}

// The same fingerprint, incrementally: fp64 is a sum of per-word terms, so a successor's
// accumulator is its parent's minus the terms of the words it changed plus their new terms
// (identical value, mod 2^64).  FpBase holds one parent's terms; successors that change few
// words skip most of the multiplies.
template <int NW32>
struct FpBase {
  static constexpr int NW64 = (NW32 + 1) / 2;
  u64 term[NW64];
  u64 sum;
  RMC_HD static u64 word(const u32 (&w)[NW32], int k) {
    return (u64)w[2 * k] | (2 * k + 1 < NW32 ? (u64)w[2 * k + 1] << 32 : 0ull);
  }
  RMC_HD static u64 key(u64 seed, int k) { return seed + (u64)(k + 1) * P1; }
  RMC_HD void init(const u32 (&w)[NW32], u64 seed) {
    sum = 0;
#pragma unroll
    for (int k = 0; k < NW64; ++k) { term[k] = fmix64(word(w, k) ^ key(seed, k)); sum += term[k]; }
  }
  // fp64(w, seed) given the parent's words `base` (from which init() was computed)
  RMC_HD u64 fp(const u32 (&w)[NW32], const u32 (&base)[NW32], u64 seed) const {
    bool changed;
    return fp(w, base, seed, changed);
  }
  // ... and whether w differs from base at all (false: the successor is its parent)
  RMC_HD u64 fp(const u32 (&w)[NW32], const u32 (&base)[NW32], u64 seed, bool& changed) const {
    u64 acc = sum;
    changed = false;
#pragma unroll
    for (int k = 0; k < NW64; ++k) {
      const u64 v = word(w, k);
      const bool d = v != word(base, k);
      changed |= d;
      if (d) acc += fmix64(v ^ key(seed, k)) - term[k];
    }
    return fp_final<NW32>(acc, seed);
  }
  // fp(w, base, seed, changed) when w can differ from base only in the 64-bit words [K0, NW64)
  // (compile-time: a successor that changes a known tail of the packed state, e.g. the message bag)
  template <int K0>
  RMC_HD u64 fp_tail(const u32 (&w)[NW32], const u32 (&base)[NW32], u64 seed, bool& changed) const {
    u64 acc = sum;
    changed = false;
#pragma unroll
    for (int k = K0; k < NW64; ++k) {
      const u64 v = word(w, k);
      const bool d = v != word(base, k);
      changed |= d;
      if (d) acc += fmix64(v ^ key(seed, k)) - term[k];
    }
    return fp_final<NW32>(acc, seed);
  }
  // fp64 of the parent's words `base` plus d * 2^P (P a compile-time bit offset into the packed
  // state, d = +-1): the successor that changes one small field by one, where the field does not
  // carry out of its own bits (so at most the two 64-bit words holding bits P.. change)
  template <int P>
  RMC_HD u64 fp_add_bit(const u32 (&base)[NW32], int d, u64 seed) const {
    constexpr int K = P >> 6, B = P & 63;
    const u64 lo = word(base, K);
    const u64 nlo = d > 0 ? lo + (1ull << B) : lo - (1ull << B);
    u64 acc = sum - term[K] + fmix64(nlo ^ key(seed, K));
    if constexpr (K + 1 < NW64) {   // a carry / borrow into the next word (the field straddles it)
      const bool c = d > 0 ? nlo < lo : nlo > lo;
      if (c) {
        const u64 hi = word(base, K + 1), nhi = d > 0 ? hi + 1 : hi - 1;
        acc += fmix64(nhi ^ key(seed, K + 1)) - term[K + 1];
      }
    }
    return fp_final<NW32>(acc, seed);
  }
};

// Compile-time bit-stream writer/reader over a u32 word array (offsets are
// template-constant after unrolling, so every access is a shift/or pair).
template <int NW32>
struct BitOut {
  u32 w[NW32];
  int pos;
  RMC_HD BitOut() : pos(0) {
#pragma unroll
    for (int k = 0; k < NW32; ++k) w[k] = 0;
  }
  RMC_HD void put(u64 v, int nb) {
    // v < 2^nb is required (callers mask)
    int q = pos >> 5, r = pos & 31;
#pragma unroll
    for (int k = 0; k < NW32; ++k) {
      if (k == q) w[k] |= (u32)(v << r);
      if (k == q + 1 && r + nb > 32) w[k] |= (u32)(v >> (32 - r));
      if (k == q + 2 && r + nb > 64) w[k] |= (u32)(v >> (64 - r));
    }
    pos += nb;
  }
};
template <int NW32>
struct BitIn {
  const u32 (&w)[NW32];
  int pos;
  RMC_HD explicit BitIn(const u32 (&words)[NW32]) : w(words), pos(0) {}
  RMC_HD u64 get(int nb) {
    // select-based (no pointer arithmetic into the register array => no scratch)
    const int q = pos >> 5, r = pos & 31;
    u64 lo = 0, mid = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < NW32; ++k) {
      if (k == q) lo = w[k];
      if (k == q + 1) mid = w[k];
      if (k == q + 2) hi = w[k];
    }
    u64 v = lo >> r;
    if (r + nb > 32) v |= mid << (32 - r);
    if (r + nb > 64) v |= hi << (64 - r);
    pos += nb;
    return v & lomask(nb);
  }
};

}  // namespace rmc
