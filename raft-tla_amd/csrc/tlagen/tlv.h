// tlv.h — TLA+ values for the generated path (host and device, no headers needed).
//
// The SANY-subset front end (tla_front.cpp) compiles a module's Init / Next / constraints /
// invariants into C++ over this library; the same text is compiled by hiprtc for gfx950 (the
// BFS kernels in tlagen_kernels.h) and by a host compiler for the CPU-side semantics tests.
//
// A value is a canonical word string in a per-thread arena, addressed by its word offset:
//   word 0: tag (3 bits) | total words << 3
//   BOOL [h, b]   INT [h, v ^ 0x80000000]   ATOM [h, id] (model values and strings, interned)
//   SEQ  [h, n, e1 .. en]                   a function whose domain is 1..n (tuples, records
//                                           never: their domain is a set of atoms)
//   FUN  [h, n, k1 v1 .. kn vn]             keys strictly increasing, domain not 1..n
//   SET  [h, n, e1 .. en]                   elements strictly increasing
// Equal TLA+ values have equal word strings (TLC's value equality: <<a, b>> = [i \in 1..2 |->
// ..], [x \in {} |-> e] = <<>>, 1 :> v = <<v>>), so a state's words are its canonical key and
// the fingerprint is a hash of the words.  Sets and function domains are kept sorted in TLC's
// value order (ocmp below: the order TLC enumerates `\E x \in S`, CHOOSE and DOMAIN in, so the
// successors come out in TLC's order); any total order would give canonical words.
//
// Errors (TLC's evaluation errors: a function applied outside its domain, a bad sequence index,
// CHOOSE with no witness, a type error, arena overflow) set bits in Ar::err and return a valid
// dummy value, so evaluation never faults; the engine reports the error for the parent state.
#pragma once
#ifndef TLV_HD
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define TLV_HD __host__ __device__ inline
#define TLV_NI __host__ __device__ __attribute__((noinline))   // large routines: one copy, not one per use
#else
#define TLV_HD inline
#define TLV_NI static __attribute__((noinline))
#endif
#endif
#ifndef TLV_CONST
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define TLV_CONST __device__ constexpr
#else
#define TLV_CONST constexpr
#endif
#endif

namespace tlv {
typedef unsigned int u32;
typedef unsigned long long u64;
typedef long long i64;

enum : u32 { T_BOOL = 1, T_INT = 2, T_ATOM = 3, T_SEQ = 4, T_FUN = 5, T_SET = 6 };
enum : u32 {
  E_OVF = 1u,        // arena or handle stack full (capacity, not a spec error)
  E_DOMAIN = 2u,     // f[x] with x outside DOMAIN f, r.fld missing
  E_TYPE = 4u,       // operand of the wrong kind
  E_CHOOSE = 8u,     // CHOOSE without a witness
  E_SEQ = 16u,       // SubSeq / Head / Tail / index out of range
  E_ASSIGN = 32u,    // x' read before it is determined
  E_ARITH = 64u,     // integer overflow / division by zero
  E_UNSUP = 128u     // construct outside the compiled subset reached at run time
};

struct Ar {
  u32* w;       // values grow up from 4 (0: FALSE, 2: TRUE)
  u32 top, cap;
  u32* hs;      // handle stack (builders)
  u32 htop, hcap;
  u32 err;
  const u32* akey;   // per atom id: AK_MV bit for model values, then its rank in TLC's order (generated)
  u32 nakey;
  u32 rdepth;        // calls of recursive function definitions in progress (bounded: kMaxRecDepth)
};
// deepest recursion of a recursive function definition a lane evaluates (deeper: E_UNSUP).  The
// kernels' stack is sized for it (tlagen_backend.cpp kRecStackBytes).
constexpr u32 kMaxRecDepth = 48;
enum : u32 { AK_MV = 1u << 30 };

TLV_HD u32 hdr(u32 tag, u32 n) { return tag | (n << 3); }
TLV_HD u32 tg(const Ar& a, u32 v) { return a.w[v] & 7u; }
TLV_HD u32 sz(const Ar& a, u32 v) { return a.w[v] >> 3; }
TLV_HD void init(Ar& a, u32* w, u32 cap, u32* hs, u32 hcap) {
  a.w = w; a.cap = cap; a.hs = hs; a.hcap = hcap; a.htop = 0; a.err = 0; a.akey = nullptr; a.nakey = 0; a.rdepth = 0;
  w[0] = hdr(T_BOOL, 2); w[1] = 0; w[2] = hdr(T_BOOL, 2); w[3] = 1; a.top = 4;
}
TLV_HD u32 alloc(Ar& a, u32 n) {
  if (a.err & E_OVF) return 0;
  if (a.top + n > a.cap) { a.err |= E_OVF; return 0; }
  const u32 r = a.top; a.top += n; return r;
}
TLV_HD void hpush(Ar& a, u32 h) { if (a.htop < a.hcap) a.hs[a.htop++] = h; else a.err |= E_OVF; }
TLV_NI u32 copy_in(Ar& a, const u32* src) {   // a value from outside the arena (state store)
  const u32 n = src[0] >> 3, r = alloc(a, n);
  if (a.err & E_OVF) return 0;
  for (u32 q = 0; q < n; ++q) a.w[r + q] = src[q];
  return r;
}

// ---- scalars
TLV_HD u32 mk_bool(bool b) { return b ? 2u : 0u; }
TLV_HD u32 mk_int(Ar& a, i64 x) {
  if (x > 2147483647LL || x < -2147483648LL) { a.err |= E_ARITH; x = 0; }
  const u32 r = alloc(a, 2);
  if (a.err & E_OVF) return 0;
  a.w[r] = hdr(T_INT, 2); a.w[r + 1] = (u32)(int)x ^ 0x80000000u; return r;
}
TLV_HD u32 mk_atom(Ar& a, u32 id) {
  const u32 r = alloc(a, 2);
  if (a.err & E_OVF) return 0;
  a.w[r] = hdr(T_ATOM, 2); a.w[r + 1] = id; return r;
}
TLV_HD i64 ival(Ar& a, u32 v) {
  if (tg(a, v) != T_INT) { a.err |= E_TYPE; return 0; }
  return (i64)(int)(a.w[v + 1] ^ 0x80000000u);
}
TLV_HD bool truth(Ar& a, u32 v) {
  if (tg(a, v) != T_BOOL) { a.err |= E_TYPE; return false; }
  return a.w[v + 1] != 0;
}

// ---- order / equality (word-lexicographic; the header holds tag and size)
TLV_NI int cmpv(const Ar& a, u32 x, u32 y) {
  if (x == y) return 0;
  const u32 n = sz(a, x) < sz(a, y) ? sz(a, x) : sz(a, y);
  for (u32 q = 0; q < n; ++q) {
    const u32 p = a.w[x + q], r = a.w[y + q];
    if (p != r) return p < r ? -1 : 1;
  }
  return 0;   // equal headers imply equal sizes
}
TLV_HD bool eqv(const Ar& a, u32 x, u32 y) {
  if (x == y) return true;
  const u32 n = sz(a, x);
  if (a.w[x] != a.w[y]) return false;
  for (u32 q = 1; q < n; ++q) if (a.w[x + q] != a.w[y + q]) return false;
  return true;
}

// ---- element walk: first element (SET/SEQ) or key (FUN) of a collection, next value
TLV_HD u32 count(const Ar& a, u32 v) { return a.w[v + 1]; }
TLV_HD u32 first(u32 v) { return v + 2; }
TLV_HD u32 nextv(const Ar& a, u32 e) { return e + sz(a, e); }
TLV_HD bool is_coll(const Ar& a, u32 v) { const u32 t = tg(a, v); return t == T_SEQ || t == T_FUN || t == T_SET; }

// TLC's value order (the oracle's cmp, oracle/tla.h:150, as TLC's Value.compareTo is recalled,
// SURVEY.md [ext]): kinds BOOLEAN < integers < strings < model values < sequences < sets <
// functions (records are functions); integers numerically, strings by text and model values by
// declaration (the atom's rank, a.akey), sequences and sets by length then element by element,
// functions by domain size, then the domain elements, then the values.  Iterative (an explicit
// stack of the collections being compared): no recursion on the device.
TLV_HD u32 orank(const Ar& a, u32 v) {
  const u32 t = tg(a, v);
  if (t == T_BOOL) return 0;
  if (t == T_INT) return 1;
  if (t == T_ATOM) { const u32 id = a.w[v + 1]; return (a.akey && id < a.nakey && (a.akey[id] & AK_MV)) ? 3 : 2; }
  return t == T_SEQ ? 4 : t == T_SET ? 5 : 6;
}
TLV_NI int ocmp(const Ar& a, u32 x, u32 y) {
  struct Fr { u32 x, y, x0, y0, left, n, fun; };   // fun: 0 SEQ/SET, 1 FUN keys, 2 FUN values
  Fr st[24];
  int sp = -1;
  u32 cx = x, cy = y;
  for (;;) {
    if (cx != cy) {
      const u32 rx = orank(a, cx), ry = orank(a, cy);
      if (rx != ry) return rx < ry ? -1 : 1;
      const u32 t = tg(a, cx);
      if (t == T_BOOL || t == T_INT) {
        const u32 p = a.w[cx + 1], q = a.w[cy + 1];
        if (p != q) return p < q ? -1 : 1;   // biased integers compare as unsigned words
      } else if (t == T_ATOM) {
        const u32 i = a.w[cx + 1], j = a.w[cy + 1];
        const u32 p = (a.akey && i < a.nakey) ? a.akey[i] : i, q = (a.akey && j < a.nakey) ? a.akey[j] : j;
        if (p != q) return p < q ? -1 : 1;
      } else {
        const u32 n = count(a, cx), m = count(a, cy);
        if (n != m) return n < m ? -1 : 1;
        if (n > 0) {
          if (sp + 1 >= 24) return cmpv(a, cx, cy);   // (nesting deeper than any spec value: word order)
          st[++sp] = Fr{first(cx), first(cy), first(cx), first(cy), n, n, t == T_FUN ? 1u : 0u};
          cx = first(cx); cy = first(cy);
          continue;
        }
      }
    }
    // the pair is equal: the next pair of the innermost collection still being compared
    for (;;) {
      if (sp < 0) return 0;
      Fr& f = st[sp];
      if (--f.left > 0) {
        f.x = nextv(a, f.x); f.y = nextv(a, f.y);
        if (f.fun) { f.x = nextv(a, f.x); f.y = nextv(a, f.y); }   // over the value (or the key)
        cx = f.x; cy = f.y;
        break;
      }
      if (f.fun == 1) {   // the domains are equal: now the values, in domain order
        f.fun = 2; f.left = f.n;
        f.x = nextv(a, f.x0); f.y = nextv(a, f.y0);
        cx = f.x; cy = f.y;
        break;
      }
      --sp;
    }
  }
}

// ---- builders: push element handles, then end
TLV_NI void sort_handles(Ar& a, u32 mark, u32 stride) {   // insertion sort of stride-groups by their first handle
  for (u32 i = mark + stride; i < a.htop; i += stride) {
    for (u32 j = i; j > mark && ocmp(a, a.hs[j - stride], a.hs[j]) > 0; j -= stride)
      for (u32 s = 0; s < stride; ++s) { const u32 t = a.hs[j - stride + s]; a.hs[j - stride + s] = a.hs[j + s]; a.hs[j + s] = t; }
  }
}
TLV_NI u32 write_coll(Ar& a, u32 tag, u32 mark, u32 stride, u32 take_from, bool dedup) {
  // writes the stride-groups hs[mark..htop) (only handles take_from.. of each group) as one value
  u32 n = 0, words = 2;
  for (u32 i = mark; i < a.htop; i += stride) {
    if (dedup && i > mark && eqv(a, a.hs[i - stride], a.hs[i])) continue;
    ++n;
    for (u32 s = take_from; s < stride; ++s) words += sz(a, a.hs[i + s]);
  }
  const u32 r = alloc(a, words);
  if (a.err & E_OVF) { a.htop = mark; return 0; }
  a.w[r] = hdr(tag, words); a.w[r + 1] = n;
  u32 o = r + 2;
  for (u32 i = mark; i < a.htop; i += stride) {
    if (dedup && i > mark && eqv(a, a.hs[i - stride], a.hs[i])) continue;
    for (u32 s = take_from; s < stride; ++s) {
      const u32 h = a.hs[i + s], m = sz(a, h);
      for (u32 q = 0; q < m; ++q) a.w[o + q] = a.w[h + q];
      o += m;
    }
  }
  a.htop = mark;
  return r;
}
TLV_HD u32 set_end(Ar& a, u32 mark) { sort_handles(a, mark, 1); return write_coll(a, T_SET, mark, 1, 0, true); }
TLV_HD u32 seq_end(Ar& a, u32 mark) { return write_coll(a, T_SEQ, mark, 1, 0, false); }
// function from (key, value) handle pairs; duplicate keys keep the first pair (callers never
// produce two values for one key: a constructor's domain is a set)
TLV_NI u32 fun_end(Ar& a, u32 mark) {
  sort_handles(a, mark, 2);
  u32 w = mark;   // drop later duplicates of a key (stable sort keeps insertion order of ties)
  for (u32 i = mark; i < a.htop; i += 2) {
    if (w > mark && eqv(a, a.hs[w - 2], a.hs[i])) continue;
    a.hs[w] = a.hs[i]; a.hs[w + 1] = a.hs[i + 1]; w += 2;
  }
  a.htop = w;
  bool seq = true;
  i64 k = 1;
  for (u32 i = mark; i < a.htop; i += 2, ++k) {
    const u32 h = a.hs[i];
    if (tg(a, h) != T_INT || (i64)(int)(a.w[h + 1] ^ 0x80000000u) != k) { seq = false; break; }
  }
  return seq ? write_coll(a, T_SEQ, mark, 2, 1, false) : write_coll(a, T_FUN, mark, 2, 0, false);
}

// ---- sets
TLV_NI bool set_in(Ar& a, u32 x, u32 s) {
  if (tg(a, s) != T_SET) { a.err |= E_TYPE; return false; }
  u32 e = first(s);
  for (u32 i = 0, n = count(a, s); i < n; ++i, e = nextv(a, e)) {
    const int c = ocmp(a, e, x);
    if (c == 0) return true;
    if (c > 0) return false;   // sorted
  }
  return false;
}
TLV_HD u32 set_card(Ar& a, u32 s) {
  if (tg(a, s) != T_SET) { a.err |= E_TYPE; return 0; }
  return count(a, s);
}
TLV_NI u32 set_union(Ar& a, u32 x, u32 y) {   // linear merge of two sorted sets
  if (tg(a, x) != T_SET || tg(a, y) != T_SET) { a.err |= E_TYPE; return x; }
  if (count(a, y) == 0) return x;
  if (count(a, x) == 0) return y;
  const u32 mark = a.htop;
  u32 e = first(x), f = first(y), i = 0, j = 0, added = 0;
  const u32 n = count(a, x), m = count(a, y);
  while (i < n || j < m) {
    int c = i == n ? 1 : j == m ? -1 : ocmp(a, e, f);
    if (c <= 0) { hpush(a, e); e = nextv(a, e); ++i; if (c == 0) { f = nextv(a, f); ++j; } }
    else { hpush(a, f); f = nextv(a, f); ++j; ++added; }
  }
  if (!added) { a.htop = mark; return x; }   // y adds nothing: x itself
  return write_coll(a, T_SET, mark, 1, 0, false);
}
TLV_HD u32 coll_card(Ar& a, u32 f) {   // Cardinality(DOMAIN f) without building the domain
  const u32 t = tg(a, f);
  if (t != T_SEQ && t != T_FUN) { a.err |= E_TYPE; return 0; }
  return count(a, f);
}
TLV_NI u32 set_filter_in(Ar& a, u32 x, u32 y, bool keep_in) {   // x \cap y (keep_in) or x \ y
  if (tg(a, x) != T_SET || tg(a, y) != T_SET) { a.err |= E_TYPE; return x; }
  const u32 mark = a.htop;
  u32 e = first(x);
  for (u32 i = 0, n = count(a, x); i < n; ++i, e = nextv(a, e))
    if (set_in(a, e, y) == keep_in) hpush(a, e);
  if (a.htop - mark == count(a, x)) { a.htop = mark; return x; }   // every element kept: x itself
  return write_coll(a, T_SET, mark, 1, 0, false);   // a subsequence of a sorted set
}
TLV_HD u32 set_cap(Ar& a, u32 x, u32 y) { return set_filter_in(a, x, y, true); }
TLV_HD u32 set_minus(Ar& a, u32 x, u32 y) { return set_filter_in(a, x, y, false); }
TLV_NI bool set_subseteq(Ar& a, u32 x, u32 y) {
  if (tg(a, x) != T_SET || tg(a, y) != T_SET) { a.err |= E_TYPE; return false; }
  u32 e = first(x);
  for (u32 i = 0, n = count(a, x); i < n; ++i, e = nextv(a, e)) if (!set_in(a, e, y)) return false;
  return true;
}
TLV_NI u32 range(Ar& a, i64 lo, i64 hi) {
  const u32 mark = a.htop;
  for (i64 k = lo; k <= hi; ++k) hpush(a, mk_int(a, k));
  return write_coll(a, T_SET, mark, 1, 0, false);
}
TLV_NI u32 powerset(Ar& a, u32 s) {
  if (tg(a, s) != T_SET) { a.err |= E_TYPE; return s; }
  const u32 n = count(a, s);
  if (n > 16) { a.err |= E_UNSUP; return s; }
  const u32 outer = a.htop;
  for (u32 m = 0; m < (1u << n); ++m) {
    const u32 mark = a.htop;
    u32 e = first(s);
    for (u32 i = 0; i < n; ++i, e = nextv(a, e)) if ((m >> i) & 1u) hpush(a, e);
    const u32 sub = write_coll(a, T_SET, mark, 1, 0, false);
    hpush(a, sub);
  }
  return set_end(a, outer);
}
TLV_NI u32 union_all(Ar& a, u32 s) {   // UNION s
  if (tg(a, s) != T_SET) { a.err |= E_TYPE; return s; }
  const u32 mark = a.htop;
  u32 e = first(s);
  for (u32 i = 0, n = count(a, s); i < n; ++i, e = nextv(a, e)) {
    if (tg(a, e) != T_SET) { a.err |= E_TYPE; continue; }
    u32 f = first(e);
    for (u32 j = 0, m = count(a, e); j < m; ++j, f = nextv(a, f)) hpush(a, f);
  }
  return set_end(a, mark);
}

// [S -> T]: every function from S to T, |T|^|S| of them (more than 2^20: E_UNSUP).  A membership test
// x \in [S -> T] never builds it (the generated code tests the domain and each value instead).
TLV_NI u32 fun_set(Ar& a, u32 s, u32 t) {
  if (tg(a, s) != T_SET || tg(a, t) != T_SET) { a.err |= E_TYPE; return s; }
  const u32 n = count(a, s), m = count(a, t);
  u64 total = 1;
  for (u32 i = 0; i < n; ++i) { total *= m; if (total > (1ull << 20)) { a.err |= E_UNSUP; return s; } }
  const u32 base = a.htop;   // the elements of S, then of T, as indexable handles
  u32 e = first(s);
  for (u32 i = 0; i < n; ++i, e = nextv(a, e)) hpush(a, e);
  e = first(t);
  for (u32 j = 0; j < m; ++j, e = nextv(a, e)) hpush(a, e);
  if (a.err & E_OVF) { a.htop = base; return s; }
  const u32 outer = a.htop;
  for (u64 idx = 0; idx < total; ++idx) {
    const u32 mark = a.htop;
    u64 r = idx;
    for (u32 i = 0; i < n; ++i, r /= m) { hpush(a, a.hs[base + i]); hpush(a, a.hs[base + n + (u32)(r % m)]); }
    const u32 f = fun_end(a, mark);
    hpush(a, f);
  }
  const u32 res = set_end(a, outer);
  a.htop = base;
  return res;
}
// [f1 : S1, ..., fk : Sk] from (field atom, set) handle pairs hs[mark..htop): every record with field
// fi in Si (more than 2^20: E_UNSUP)
TLV_NI u32 rec_set(Ar& a, u32 mark) {
  const u32 k = (a.htop - mark) / 2;
  u64 total = 1;
  for (u32 i = 0; i < k; ++i) {
    const u32 si = a.hs[mark + 2 * i + 1];
    if (tg(a, si) != T_SET) { a.err |= E_TYPE; a.htop = mark; return 0; }
    total *= count(a, si);
    if (total > (1ull << 20)) { a.err |= E_UNSUP; a.htop = mark; return 0; }
  }
  const u32 outer = a.htop;
  for (u64 idx = 0; idx < total; ++idx) {
    const u32 m2 = a.htop;
    u64 r = idx;
    for (u32 i = 0; i < k; ++i) {
      const u32 si = a.hs[mark + 2 * i + 1], c = count(a, si);
      u32 e = first(si);
      for (u32 q = (u32)(r % c); q > 0; --q) e = nextv(a, e);
      r /= c;
      hpush(a, a.hs[mark + 2 * i]); hpush(a, e);
    }
    const u32 f = fun_end(a, m2);
    hpush(a, f);
  }
  const u32 res = set_end(a, outer);
  a.htop = mark;
  return res;
}

// ---- functions, records, sequences
TLV_NI u32 dom(Ar& a, u32 f) {
  const u32 t = tg(a, f);
  if (t == T_SEQ) return range(a, 1, count(a, f));
  if (t != T_FUN) { a.err |= E_TYPE; return f; }
  const u32 mark = a.htop;
  u32 e = first(f);
  for (u32 i = 0, n = count(a, f); i < n; ++i) { hpush(a, e); e = nextv(a, e); e = nextv(a, e); }
  return write_coll(a, T_SET, mark, 1, 0, false);
}
// pointer to f[x] or 0 if x is outside DOMAIN f (no error flagged)
TLV_NI u32 lookup(Ar& a, u32 f, u32 x) {
  const u32 t = tg(a, f);
  if (t == T_SEQ) {
    if (tg(a, x) != T_INT) return 0;
    const i64 k = ival(a, x);
    if (k < 1 || k > (i64)count(a, f)) return 0;
    u32 e = first(f);
    for (i64 i = 1; i < k; ++i) e = nextv(a, e);
    return e;
  }
  if (t != T_FUN) { a.err |= E_TYPE; return 0; }
  u32 e = first(f);
  for (u32 i = 0, n = count(a, f); i < n; ++i) {
    const u32 v = nextv(a, e);
    if (eqv(a, e, x)) return v;
    e = nextv(a, v);
  }
  return 0;
}
TLV_HD bool in_dom(Ar& a, u32 f, u32 x) { return lookup(a, f, x) != 0; }
TLV_HD u32 apply(Ar& a, u32 f, u32 x) {
  const u32 r = lookup(a, f, x);
  if (!r) { a.err |= E_DOMAIN; return 0; }
  return r;
}
TLV_HD u32 fun_len(Ar& a, u32 f) {   // Len
  if (tg(a, f) != T_SEQ) { a.err |= E_TYPE; return 0; }
  return count(a, f);
}
// [f EXCEPT ![x] = v]; x outside DOMAIN f leaves f unchanged (TLC)
TLV_NI u32 except(Ar& a, u32 f, u32 x, u32 v) {
  const u32 t = tg(a, f);
  if (t != T_SEQ && t != T_FUN) { a.err |= E_TYPE; return f; }
  const u32 at = lookup(a, f, x);
  if (!at) return f;
  if (eqv(a, at, v)) return f;   // the same value: f itself (no copy; the successor shows the variable unchanged)
  const u32 old = sz(a, at), nw = sz(a, v), total = sz(a, f) - old + nw;
  const u32 r = alloc(a, total);
  if (a.err & E_OVF) return 0;
  u32 o = r;
  for (u32 q = f; q < at; ++q) a.w[o++] = a.w[q];
  for (u32 q = 0; q < nw; ++q) a.w[o++] = a.w[v + q];
  for (u32 q = at + old; q < f + sz(a, f); ++q) a.w[o++] = a.w[q];
  a.w[r] = hdr(t, total);
  return r;
}
TLV_HD u32 colon_gt(Ar& a, u32 k, u32 v) {   // k :> v
  const u32 mark = a.htop;
  hpush(a, k); hpush(a, v);
  return fun_end(a, mark);
}
TLV_NI void push_pairs(Ar& a, u32 f) {
  const u32 t = tg(a, f);
  if (t == T_SEQ) {
    u32 e = first(f);
    for (u32 i = 0, n = count(a, f); i < n; ++i, e = nextv(a, e)) { hpush(a, mk_int(a, (i64)i + 1)); hpush(a, e); }
  } else if (t == T_FUN) {
    u32 e = first(f);
    for (u32 i = 0, n = count(a, f); i < n; ++i) { const u32 v = nextv(a, e); hpush(a, e); hpush(a, v); e = nextv(a, v); }
  } else a.err |= E_TYPE;
}
TLV_NI u32 atat(Ar& a, u32 f, u32 g) {   // f @@ g: f's pairs, then g's keys not in DOMAIN f
  const u32 mark = a.htop;
  push_pairs(a, f);
  push_pairs(a, g);
  return fun_end(a, mark);   // stable: f's pair wins a shared key
}
// ---- TLC's SYMMETRY: Permutations(S) and the renaming of a value by one permutation
// Permutations(S) (the TLC module): every bijection S -> S, as functions; |S| <= 6 (720 of them)
TLV_NI u32 permutations(Ar& a, u32 s) {
  if (tg(a, s) != T_SET) { a.err |= E_TYPE; return s; }
  const u32 n = count(a, s);
  if (n > 6) { a.err |= E_UNSUP; return s; }
  u32 el[6];
  u32 e = first(s);
  for (u32 i = 0; i < n; ++i, e = nextv(a, e)) el[i] = e;
  u32 idx[6];
  for (u32 i = 0; i < n; ++i) idx[i] = i;
  const u32 outer = a.htop;
  for (;;) {   // lexicographic enumeration of index permutations
    const u32 mark = a.htop;
    for (u32 i = 0; i < n; ++i) { hpush(a, el[i]); hpush(a, el[idx[i]]); }
    hpush(a, fun_end(a, mark));
    int k = (int)n - 2;
    while (k >= 0 && idx[k] > idx[k + 1]) --k;
    if (k < 0) break;
    int l = (int)n - 1;
    while (idx[l] < idx[k]) --l;
    u32 t = idx[k]; idx[k] = idx[l]; idx[l] = t;
    for (int x = k + 1, y = (int)n - 1; x < y; ++x, --y) { t = idx[x]; idx[x] = idx[y]; idx[y] = t; }
  }
  return set_end(a, outer);
}
// v with every atom in DOMAIN pi renamed to pi[atom] (sets and function domains re-sorted); a
// value that contains no renamed atom comes back as the same handle (nothing is rebuilt).
// Iterative over an explicit stack of collections being rebuilt: a recursive device function
// makes the kernel's stack size dynamic, and the GPU's default per-lane stack does not hold a
// state's nesting (messages -> record -> log -> entry ...).
TLV_NI u32 perm_value(Ar& a, u32 v, u32 pi) {
  struct Fr { u32 v, left, e, mark, changed; };   // left: element handles still to visit
  constexpr int D = 24;
  Fr st[D];
  int sp = 0;
  u32 x = v;   // the value to rename next
  for (;;) {
    const u32 t = tg(a, x);
    u32 r = x;   // x renamed, once known
    bool done = true;
    if (t == T_ATOM) {
      const u32 q = lookup(a, pi, x);
      r = q ? q : x;
    } else if (t == T_SEQ || t == T_FUN || t == T_SET) {
      const u32 n = count(a, x) * (t == T_FUN ? 2u : 1u);
      if (n > 0) {
        if (sp == D) { a.err |= E_UNSUP; return v; }   // (nesting deeper than any spec value)
        st[sp++] = Fr{x, n, first(x), a.htop, 0u};
        x = first(x);
        done = false;
      }
    }
    if (!done) continue;
    // r is the renamed x: hand it to the enclosing collections, closing each that is complete
    for (;;) {
      if (sp == 0) return r;
      Fr& f = st[sp - 1];
      f.changed |= r != f.e ? 1u : 0u;
      hpush(a, r);
      if (--f.left > 0) { f.e = nextv(a, f.e); x = f.e; break; }
      const u32 tf = tg(a, f.v);
      if (!f.changed) { a.htop = f.mark; r = f.v; }
      else r = tf == T_SET ? set_end(a, f.mark) : tf == T_FUN ? fun_end(a, f.mark) : seq_end(a, f.mark);
      --sp;
    }
  }
}

// ---- the standard Bags module (a bag: a function from elements to positive counts)
TLV_NI u32 set_to_bag(Ar& a, u32 s) {   // SetToBag(S) == [e \in S |-> 1]
  if (tg(a, s) != T_SET) { a.err |= E_TYPE; return s; }
  const u32 mark = a.htop;
  u32 e = first(s);
  for (u32 i = 0, n = count(a, s); i < n; ++i, e = nextv(a, e)) { hpush(a, e); hpush(a, mk_int(a, 1)); }
  return fun_end(a, mark);
}
TLV_NI u32 bag_op(Ar& a, u32 x, u32 y, bool add) {   // B1 (+) B2, B1 (-) B2 (counts <= 0 leave the domain)
  const u32 tx = tg(a, x), ty = tg(a, y);
  if ((tx != T_SEQ && tx != T_FUN) || (ty != T_SEQ && ty != T_FUN)) { a.err |= E_TYPE; return x; }
  const u32 pm = a.htop;
  push_pairs(a, x);
  const u32 px = a.htop;
  push_pairs(a, y);
  const u32 py = a.htop;
  const u32 mark = a.htop;
  for (u32 i = pm; i < px; i += 2) {
    const u32 k = a.hs[i];
    i64 c = ival(a, a.hs[i + 1]);
    const u32 o = lookup(a, y, k);
    if (o) c += add ? ival(a, o) : -ival(a, o);
    if (c > 0) { hpush(a, k); hpush(a, mk_int(a, c)); }
  }
  if (add)
    for (u32 i = px; i < py; i += 2)
      if (!lookup(a, x, a.hs[i])) { hpush(a, a.hs[i]); hpush(a, a.hs[i + 1]); }
  // move the result pairs down over the operands' pairs, then build
  u32 w = pm;
  for (u32 i = mark; i < a.htop; ++i) a.hs[w++] = a.hs[i];
  a.htop = w;
  return fun_end(a, pm);
}
TLV_NI i64 bag_card(Ar& a, u32 b) {   // BagCardinality
  const u32 t = tg(a, b);
  if (t != T_SEQ && t != T_FUN) { a.err |= E_TYPE; return 0; }
  i64 s = 0;
  u32 e = first(b);
  for (u32 i = 0, n = count(a, b); i < n; ++i) {
    if (t == T_FUN) e = nextv(a, e);   // skip the key
    s += ival(a, e);
    e = nextv(a, e);
  }
  return s;
}

TLV_NI u32 append(Ar& a, u32 s, u32 e) {
  if (tg(a, s) != T_SEQ) { a.err |= E_TYPE; return s; }
  const u32 n = sz(a, s), m = sz(a, e), r = alloc(a, n + m);
  if (a.err & E_OVF) return 0;
  for (u32 q = 0; q < n; ++q) a.w[r + q] = a.w[s + q];
  for (u32 q = 0; q < m; ++q) a.w[r + n + q] = a.w[e + q];
  a.w[r] = hdr(T_SEQ, n + m); a.w[r + 1] = count(a, s) + 1;
  return r;
}
TLV_NI u32 concat(Ar& a, u32 s, u32 t) {   // s \o t
  if (tg(a, s) != T_SEQ || tg(a, t) != T_SEQ) { a.err |= E_TYPE; return s; }
  const u32 n = sz(a, s), m = sz(a, t) - 2, r = alloc(a, n + m);
  if (a.err & E_OVF) return 0;
  for (u32 q = 0; q < n; ++q) a.w[r + q] = a.w[s + q];
  for (u32 q = 0; q < m; ++q) a.w[r + n + q] = a.w[t + 2 + q];
  a.w[r] = hdr(T_SEQ, n + m); a.w[r + 1] = count(a, s) + count(a, t);
  return r;
}
TLV_NI u32 subseq(Ar& a, u32 s, i64 m, i64 n) {   // SubSeq(s, m, n)
  if (tg(a, s) != T_SEQ) { a.err |= E_TYPE; return s; }
  const u32 mark = a.htop;
  if (m > n) return seq_end(a, mark);
  if (m < 1 || n > (i64)count(a, s)) { a.err |= E_SEQ; return seq_end(a, mark); }
  u32 e = first(s);
  for (i64 i = 1; i <= n; ++i, e = nextv(a, e)) if (i >= m) hpush(a, e);
  return seq_end(a, mark);
}
TLV_HD u32 head(Ar& a, u32 s) {
  if (tg(a, s) != T_SEQ || count(a, s) == 0) { a.err |= E_SEQ; return 0; }
  return first(s);
}
TLV_HD u32 tail(Ar& a, u32 s) {
  if (tg(a, s) != T_SEQ || count(a, s) == 0) { a.err |= E_SEQ; return s; }
  return subseq(a, s, 2, count(a, s));
}

// ---- state words and fingerprint
TLV_HD u64 fmix(u64 h) { h ^= h >> 33; h *= 0xff51afd7ed558ccdULL; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ULL; h ^= h >> 33; return h; }
TLV_NI u64 fp_words(const u32* w, u32 n, u64 seed) {
  u64 h = seed ^ ((u64)n * 0x9e3779b97f4a7c15ULL);
  u32 q = 0;
  for (; q + 1 < n; q += 2) h = fmix(h ^ (((u64)w[q + 1] << 32) | w[q])) + 0x9e3779b97f4a7c15ULL;
  if (q < n) h = fmix(h ^ (u64)w[q] ^ 0x5555555500000000ULL);
  h = fmix(h);
  return h ? h : 1ULL;   // 0 marks an empty seen-set slot
}
}  // namespace tlv
