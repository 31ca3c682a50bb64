// Python's repr(float) -- the text json.dumps writes for a score -- as __host__ __device__ code,
// so the score files' doubles are formatted on the GPU (repr.hip) and the same function is
// checked against CPython's repr on the CPU (tests/test_repr.py).
//
// Digits: the shortest decimal that reads back as v, closest to v among the shortest, ties to
// even -- what CPython's dtoa mode 0 returns. The search follows Ryu (U. Adams, PLDI 2018): the
// interval of reals that round to v, [4m - 1 - s, 4m + 2] * 2^(e2), is scaled by 10^-q with a
// 125-bit fixed-point power of five (repr_tables.h), and decimal digits are dropped while the
// interval's ends still differ in the remaining prefix; exact-tie bookkeeping (trailing zeros
// of the scaled ends) decides the last digit. Layout: CPython's float_repr_style 'short' with
// Py_DTSF_ADD_DOT_0 -- fixed notation for a decimal point position in (-4, 16], else
// d[.ddd]e(+|-)XX; integral values end in ".0".
#pragma once
#include <stdint.h>

#include "repr_tables.h"

namespace blp {

constexpr int REPR_SLOT = 24;  // the longest repr: "-2.2250738585072014e-308"

struct ReprTables {
  const uint64_t* p5;   // [BLP_REPR_N_P5][2]
  const uint64_t* inv;  // [BLP_REPR_N_INV][2]
};

__host__ __device__ inline int32_t repr_pow5bits(int32_t e) { return ((e * 1217359) >> 19) + 1; }
__host__ __device__ inline int32_t repr_log10pow2(int32_t e) { return (e * 78913) >> 18; }
__host__ __device__ inline int32_t repr_log10pow5(int32_t e) { return (e * 732923) >> 20; }

__host__ __device__ inline bool repr_mul_pow5(uint64_t v, int32_t p) {  // 5^p | v (v > 0)
  int32_t c = 0;
  while (v % 5 == 0) {
    v /= 5;
    ++c;
  }
  return c >= p;
}

// (m * w) >> j for the 125-bit w = {lo, hi} and j >= 64
__host__ __device__ inline uint64_t repr_mulshift(uint64_t m, const uint64_t* w, int32_t j) {
  const unsigned __int128 lo = (unsigned __int128)m * w[0];
  const unsigned __int128 hi = (unsigned __int128)m * w[1];
  return (uint64_t)(((lo >> 64) + hi) >> (j - 64));
}

// v = digits * 10^exp10, digits the shortest round-trip decimal of a finite, nonzero |v|
__host__ __device__ inline void repr_shortest(uint64_t frac, int32_t bexp, const ReprTables& t, uint64_t* digits,
                                              int32_t* exp10) {
  int32_t e2;
  uint64_t m2;
  if (bexp == 0) {
    e2 = 1 - 1023 - 52 - 2;
    m2 = frac;
  } else {
    e2 = bexp - 1023 - 52 - 2;
    m2 = (1ull << 52) | frac;
  }
  const bool accept = (m2 & 1) == 0;  // round-half-even reads the interval's ends back as v
  const uint64_t mv = 4 * m2;
  const uint32_t mm_shift = (frac != 0 || bexp <= 1) ? 1u : 0u;  // the lower gap halves at a binade
  uint64_t vr, vp, vm;
  int32_t e10;
  bool vm_tz = false, vr_tz = false;  // the scaled ends are exact (only zeros dropped)
  if (e2 >= 0) {
    const int32_t q = repr_log10pow2(e2) - (e2 > 3 ? 1 : 0);
    e10 = q;
    const int32_t j = -e2 + q + 125 + repr_pow5bits(q) - 1;
    const uint64_t* w = t.inv + 2 * q;
    vr = repr_mulshift(mv, w, j);
    vp = repr_mulshift(mv + 2, w, j);
    vm = repr_mulshift(mv - 1 - mm_shift, w, j);
    if (q <= 21) {  // 5^q may divide the end points: exactness matters
      if (mv % 5 == 0)
        vr_tz = repr_mul_pow5(mv, q);
      else if (accept)
        vm_tz = repr_mul_pow5(mv - 1 - mm_shift, q);
      else
        vp -= repr_mul_pow5(mv + 2, q) ? 1 : 0;
    }
  } else {
    const int32_t q = repr_log10pow5(-e2) - (-e2 > 1 ? 1 : 0);
    e10 = q + e2;
    const int32_t i = -e2 - q;
    const int32_t j = q - (repr_pow5bits(i) - 125);
    const uint64_t* w = t.p5 + 2 * i;
    vr = repr_mulshift(mv, w, j);
    vp = repr_mulshift(mv + 2, w, j);
    vm = repr_mulshift(mv - 1 - mm_shift, w, j);
    if (q <= 1) {
      vr_tz = true;  // mv has >= 2 factors of two
      if (accept)
        vm_tz = mm_shift == 1;
      else
        --vp;
    } else if (q < 63) {
      vr_tz = (mv & ((1ull << q) - 1)) == 0;  // 2^q | mv (-e2 >= q supplies the fives)
    }
  }
  int32_t removed = 0;
  uint32_t last = 0;
  uint64_t out;
  if (vm_tz || vr_tz) {  // rare: a possible exact tie
    while (vp / 10 > vm / 10) {
      vm_tz &= vm % 10 == 0;
      vr_tz &= last == 0;
      last = (uint32_t)(vr % 10);
      vr /= 10;
      vp /= 10;
      vm /= 10;
      ++removed;
    }
    if (vm_tz) {
      while (vm % 10 == 0) {
        vr_tz &= last == 0;
        last = (uint32_t)(vr % 10);
        vr /= 10;
        vp /= 10;
        vm /= 10;
        ++removed;
      }
    }
    if (vr_tz && last == 5 && vr % 2 == 0) last = 4;  // exactly half way: to even
    out = vr + (((vr == vm && (!accept || !vm_tz)) || last >= 5) ? 1 : 0);
  } else {
    bool up = false;
    if (vp / 100 > vm / 100) {  // two digits at a time first
      up = vr % 100 >= 50;
      vr /= 100;
      vp /= 100;
      vm /= 100;
      removed += 2;
    }
    while (vp / 10 > vm / 10) {
      up = vr % 10 >= 5;
      vr /= 10;
      vp /= 10;
      vm /= 10;
      ++removed;
    }
    out = vr + ((vr == vm || up) ? 1 : 0);
  }
  *digits = out;
  *exp10 = e10 + removed;
}

// A repr under construction: 24 bytes in three registers (byte k of the text = byte k % 8 of
// word k / 8, little-endian as stored), NUL-padded; no dynamically indexed arrays, so the
// device code keeps it out of scratch memory.
struct Repr24 {
  uint64_t w0 = 0, w1 = 0, w2 = 0;
  int n = 0;
  __host__ __device__ inline void put(char c) {
    const uint64_t v = (uint64_t)(uint8_t)c << (8 * (n & 7));
    const int k = n >> 3;
    w0 |= k == 0 ? v : 0;
    w1 |= k == 1 ? v : 0;
    w2 |= k == 2 ? v : 0;
    ++n;
  }
};

// repr(v) -- json.dumps' text for a float -- into r. zero_int: 0.0 is written as the int 0
// (adamic_adar's "nothing added", similarity.py:118).
__host__ __device__ inline void repr_double(double v, bool zero_int, const ReprTables& t, Repr24& r) {
  const uint64_t bits = __builtin_bit_cast(uint64_t, v);
  const bool neg = (bits >> 63) != 0;
  const int32_t bexp = (int32_t)((bits >> 52) & 0x7ff);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  if (bexp == 0x7ff) {  // json.dumps: NaN, Infinity, -Infinity
    if (frac) {
      r.put('N'), r.put('a'), r.put('N');
      return;
    }
    if (neg) r.put('-');
    const char inf[] = "Infinity";
    for (int i = 0; i < 8; ++i) r.put(inf[i]);
    return;
  }
  if (bexp == 0 && frac == 0) {
    if (zero_int) {
      r.put('0');
      return;
    }
    if (neg) r.put('-');
    r.put('0'), r.put('.'), r.put('0');
    return;
  }
  uint64_t d;
  int32_t e10;
  repr_shortest(frac, bexp, t, &d, &e10);
  // the digits as BCD nibbles, least significant first (<= 17 digits: two words)
  uint64_t b0 = 0, b1 = 0;
  int nd = 0;
  for (uint64_t x = d; x; x /= 10, ++nd) {
    const uint64_t dg = x % 10;
    if (nd < 16)
      b0 |= dg << (4 * nd);
    else
      b1 |= dg << (4 * (nd - 16));
  }
  auto digit = [&](int i) -> char {  // i-th digit from the most significant
    const int k = nd - 1 - i;
    const uint64_t w = k < 16 ? b0 >> (4 * k) : b1 >> (4 * (k - 16));
    return (char)('0' + (w & 15));
  };
  const int decpt = e10 + nd;  // |v| = 0.d1d2... * 10^decpt
  if (neg) r.put('-');
  if (decpt <= -4 || decpt > 16) {
    r.put(digit(0));
    if (nd > 1) {
      r.put('.');
      for (int i = 1; i < nd; ++i) r.put(digit(i));
    }
    int e = decpt - 1;
    r.put('e');
    r.put(e < 0 ? '-' : '+');
    if (e < 0) e = -e;
    if (e >= 100) {
      r.put((char)('0' + e / 100));
      e %= 100;
    }
    r.put((char)('0' + e / 10));  // at least two exponent digits
    r.put((char)('0' + e % 10));
  } else if (decpt <= 0) {
    r.put('0');
    r.put('.');
    for (int i = 0; i < -decpt; ++i) r.put('0');
    for (int i = 0; i < nd; ++i) r.put(digit(i));
  } else if (decpt >= nd) {
    for (int i = 0; i < nd; ++i) r.put(digit(i));
    for (int i = nd; i < decpt; ++i) r.put('0');
    r.put('.');
    r.put('0');
  } else {
    for (int i = 0; i < decpt; ++i) r.put(digit(i));
    r.put('.');
    for (int i = decpt; i < nd; ++i) r.put(digit(i));
  }
}

}  // namespace blp
