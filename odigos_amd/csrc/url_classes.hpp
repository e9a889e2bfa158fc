// url_classes.hpp — the byte classes of the URL classifier's bitmaps
// (url_kernel.hip), from two nibble lookups and a bit-matrix transpose.
//
// A row of 32 staged bytes becomes one 32-bit word per class (bit k = byte k
// is in the class).  Each byte gets two 8-bit codes, each bit of a code a
// rectangle (hi-nibble set x lo-nibble set) found by ANDing two table
// lookups (v_perm_b32 picks any of 8 bytes: an 8-entry table per dword pair;
// the lo nibble's 16 entries are two lookups and a select on its bit 3).  The
// codes of 8 bytes form an 8 x 8 bit matrix whose transpose (three delta
// swaps) holds, in byte b, code bit b of the 8 bytes; a 4 x 4 byte transpose
// of the four 8-byte blocks then gives the 32-bit words.  The classes are
// boolean combinations of the rectangles.  This replaced per-class SWAR range
// tests (two compares per bound) and a shift-and-OR per class and dword: 636
// vector instructions per row before, about 360 now.
//
// The hi-nibble index keeps 3 bits, so bytes >= 0x80 alias ASCII ones: the
// high-bit plane (code P bit 7, the byte's own bit 7) masks them out.
//
// Plain functions of the bytes, compiled for the host too: tests/lut_check.cpp
// compares them with the byte predicates of templatize.go's regexps.
#pragma once
#include <cstdint>

#if defined(__HIP__)
#define OSE_UC __host__ __device__ __forceinline__
#else
#define OSE_UC inline
#endif

namespace ose {
namespace uc {

// v_perm_b32: byte i of the result is selected by byte i of sel from the
// 8 bytes {s0 (bytes 4-7), s1 (bytes 0-3)}; 8-11 sign-extend bytes 1, 3, 5,
// 7; 12 gives 0x00, 13 and above 0xFF
OSE_UC uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(s0, s1, sel);
#else
  const uint64_t v = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) {
    const uint32_t s = (sel >> (8 * i)) & 0xFFu;
    uint32_t b;
    if (s >= 13) b = 0xFFu;
    else if (s == 12) b = 0u;
    else if (s >= 8) b = ((v >> (8 * (2 * (s - 8) + 1) + 7)) & 1u) ? 0xFFu : 0u;
    else b = (uint32_t)(v >> (8 * s)) & 0xFFu;
    r |= b << (8 * i);
  }
  return r;
#endif
}

// code P: bit 0 digit {3}x{0-9}, 1 hex letter {4,6}x{1-6}, 2-3 letters
// {4,6}x{1-F} | {5,7}x{0-A}, 4-6 printable {2}x{1-F} | {3-6}x{0-F} |
// {7}x{0-E}, 7 the byte's high bit (ORed in, not looked up)
constexpr uint32_t hp_entry(uint32_t h) {
  return (h == 3 ? 0x01u : 0u) | ((h == 4 || h == 6) ? 0x06u : 0u) | ((h == 5 || h == 7) ? 0x08u : 0u) |
         (h == 2 ? 0x10u : 0u) | ((h >= 3 && h <= 6) ? 0x20u : 0u) | (h == 7 ? 0x40u : 0u);
}
constexpr uint32_t lp_entry(uint32_t l) {
  return (l <= 9 ? 0x01u : 0u) | ((l >= 1 && l <= 6) ? 0x02u : 0u) | (l >= 1 ? 0x04u : 0u) | (l <= 10 ? 0x08u : 0u) |
         (l >= 1 ? 0x10u : 0u) | 0x20u | (l <= 14 ? 0x40u : 0u);
}
// code Q (single bytes): bit 0 '-' (2,D), 1 '.' (2,E), 2 '/' (2,F), 3 '?'
// (3,F), 4 '@' (4,0), 5 '_' (5,F), 6 '%' or '+' {2}x{5,B}
constexpr uint32_t hq_entry(uint32_t h) {
  return h == 2 ? 0x47u : h == 3 ? 0x08u : h == 4 ? 0x10u : h == 5 ? 0x20u : 0u;
}
constexpr uint32_t lq_entry(uint32_t l) {
  return l == 0xD ? 0x01u : l == 0xE ? 0x02u : l == 0xF ? 0x2Cu : l == 0 ? 0x10u : (l == 5 || l == 0xB) ? 0x40u : 0u;
}
template <class F>
constexpr uint32_t tab4(F f, uint32_t base) {
  return f(base) | (f(base + 1) << 8) | (f(base + 2) << 16) | (f(base + 3) << 24);
}
constexpr uint32_t kHP0 = tab4(hp_entry, 0), kHP1 = tab4(hp_entry, 4);
constexpr uint32_t kLP0 = tab4(lp_entry, 0), kLP1 = tab4(lp_entry, 4), kLP2 = tab4(lp_entry, 8),
                   kLP3 = tab4(lp_entry, 12);
constexpr uint32_t kHQ0 = tab4(hq_entry, 0), kHQ1 = tab4(hq_entry, 4);
constexpr uint32_t kLQ0 = tab4(lq_entry, 0), kLQ1 = tab4(lq_entry, 4), kLQ2 = tab4(lq_entry, 8),
                   kLQ3 = tab4(lq_entry, 12);

// the two codes of each byte of x
OSE_UC void codes(uint32_t x, uint32_t& P, uint32_t& Q) {
  const uint32_t lo7 = x & 0x07070707u, hi = (x >> 4) & 0x07070707u;
  const uint32_t m3 = perm(0u, 0u, ((x >> 3) & 0x01010101u) | 0x0C0C0C0Cu);   // 0xFF where lo nibble >= 8
  const uint32_t pa = perm(kLP1, kLP0, lo7), pb = perm(kLP3, kLP2, lo7);
  const uint32_t qa = perm(kLQ1, kLQ0, lo7), qb = perm(kLQ3, kLQ2, lo7);
  const uint32_t hp = perm(kHP1, kHP0, hi), hq = perm(kHQ1, kHQ0, hi);
  P = (((m3 & pb) | (~m3 & pa)) & hp) | (x & 0x80808080u);
  Q = ((m3 & qb) | (~m3 & qa)) & hq;
}

// 8 x 8 bit transpose of the 64-bit {hi, lo}: bit 8i + b -> bit 8b + i
// (delta swaps of 7, 14 and 28 bit places)
OSE_UC void xpose8(uint32_t& lo, uint32_t& hi) {
  uint32_t t;
  t = (lo ^ (lo >> 7)) & 0x00AA00AAu;
  lo ^= t ^ (t << 7);
  t = (hi ^ (hi >> 7)) & 0x00AA00AAu;
  hi ^= t ^ (t << 7);
  t = (lo ^ (lo >> 14)) & 0x0000CCCCu;
  lo ^= t ^ (t << 14);
  t = (hi ^ (hi >> 14)) & 0x0000CCCCu;
  hi ^= t ^ (t << 14);
  t = (lo ^ (hi << 4)) & 0xF0F0F0F0u;
  lo ^= t;
  hi ^= t >> 4;
}

// 4 x 4 byte transpose: out[d] byte j = in[j] byte d
OSE_UC void xpose4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t* out) {
  const uint32_t t0 = perm(a1, a0, 0x05010400u);   // a0.b0 a1.b0 a0.b1 a1.b1
  const uint32_t t1 = perm(a1, a0, 0x07030602u);   // a0.b2 a1.b2 a0.b3 a1.b3
  const uint32_t t2 = perm(a3, a2, 0x05010400u);
  const uint32_t t3 = perm(a3, a2, 0x07030602u);
  out[0] = perm(t2, t0, 0x05040100u);
  out[1] = perm(t2, t0, 0x07060302u);
  out[2] = perm(t3, t1, 0x05040100u);
  out[3] = perm(t3, t1, 0x07060302u);
}

// the classifier's class order (url_kernel.hip C_*)
enum : uint32_t { BNL = 0, BHX, DG, AT, HI, DASH, SL, QM, BLOC, BDOM, DOT, NAL, kN };

// the 12 class words from the 15 code planes (p[b]: P bit b, q[b]: Q bit b);
// every ASCII plane is masked with the high-bit plane (aliased hi nibbles)
OSE_UC void derive(const uint32_t* p, const uint32_t* q, uint32_t* out) {
  const uint32_t nh = ~p[7];
  const uint32_t dg = p[0] & nh, al = (p[2] | p[3]) & nh, pr = (p[4] | p[5] | p[6]) & nh;
  const uint32_t dash = q[0] & nh, dot = q[1] & nh;
  out[BNL] = ~pr | al;                       // outside noLetters' class (templatize.go:14)
  out[BHX] = ~((p[0] | p[1]) & nh);          // outside [0-9A-Fa-f]
  out[DG] = dg;
  out[AT] = q[4] & nh;
  out[HI] = p[7];
  out[DASH] = dash;
  out[SL] = q[2] & nh;
  out[QM] = q[3] & nh;
  const uint32_t bdom = ~(al | dg | dot | dash);   // outside [A-Za-z0-9.-] (emailRegex domain)
  out[BDOM] = bdom;
  out[BLOC] = bdom & ~((q[5] | q[6]) & nh);        // outside [A-Za-z0-9._%+-] (emailRegex local part)
  out[DOT] = dot;
  out[NAL] = ~al;
}

// the class words of one 32-byte row (x[d] = bytes 4d..4d+3)
OSE_UC void row_classes(const uint32_t* x, uint32_t* out) {
  uint32_t P[8], Q[8];
  for (int d = 0; d < 8; d++) codes(x[d], P[d], Q[d]);
  for (int j = 0; j < 4; j++) {   // block j: bytes 8j..8j+7
    xpose8(P[2 * j], P[2 * j + 1]);
    xpose8(Q[2 * j], Q[2 * j + 1]);
  }
  uint32_t p[8], q[8];
  xpose4(P[0], P[2], P[4], P[6], p);       // planes 0-3: byte j from block j
  xpose4(P[1], P[3], P[5], P[7], p + 4);   // planes 4-7
  xpose4(Q[0], Q[2], Q[4], Q[6], q);
  xpose4(Q[1], Q[3], Q[5], Q[7], q + 4);
  derive(p, q, out);
}

}  // namespace uc
}  // namespace ose
