// url_classes.hpp — the byte classes of the URL classifier's bitmaps
// (url_kernel.hip), bit-sliced.
//
// A row of 32 staged bytes becomes one 32-bit word per class (bit k = byte k
// is in the class).  The row's raw bytes are transposed into their 8 bit
// planes (plane b, bit k = bit b of byte k): an 8 x 8 bit transpose of each
// 8-byte block (three delta swaps) puts bit b of the block's 8 bytes in its
// byte b, and a 4 x 4 byte transpose of the four blocks gives the 32-bit
// planes.  Every class is then a boolean function of the 8 planes, evaluated
// for the 32 bytes at once (hi-nibble and lo-nibble minterms shared between
// the classes): exact for all 256 byte values, no lookup tables.  About 200
// vector instructions per row; the round-4 form (two nibble-lookup codes per
// byte and twice the transposes) took about 470, the round-3 per-class SWAR
// range tests 636.
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

// the 12 class words from the 8 bit planes b[0..7] of 32 bytes
OSE_UC void derive_planes(const uint32_t* b, uint32_t* out) {
  const uint32_t A = ~b[7];   // ASCII
  // hi nibble (bits 6-4) of ASCII bytes
  const uint32_t m6 = A & b[6], z6 = A & ~b[6];
  const uint32_t h01 = z6 & ~b[5];
  const uint32_t h2 = z6 & b[5] & ~b[4], h3 = z6 & b[5] & b[4];
  const uint32_t h46 = m6 & ~b[4], h57 = m6 & b[4];                 // 0x4_ | 0x6_, 0x5_ | 0x7_
  const uint32_t h4 = h46 & ~b[5], h5 = h57 & ~b[5], h7 = h57 & b[5];
  // lo nibble
  const uint32_t nz = b[3] | b[2] | b[1] | b[0];                    // lo != 0
  const uint32_t le9 = ~b[3] | ~(b[2] | b[1]);                     // 0-9
  const uint32_t le10 = ~b[3] | ~(b[2] | (b[1] & b[0]));           // 0-10
  const uint32_t c3 = b[3] & b[2];                                  // 0xC-0xF
  const uint32_t lF = c3 & b[1] & b[0], lE = c3 & b[1] & ~b[0], lD = c3 & ~b[1] & b[0];
  const uint32_t l16 = ~b[3] & nz & ~(b[2] & b[1] & b[0]);          // 1-6
  const uint32_t l5B = b[0] & (b[3] ^ b[2]) & (b[1] ^ b[2]);       // 5 (0101) or 0xB (1011)
  const uint32_t dg = h3 & le9;
  const uint32_t al = (h46 & nz) | (h57 & le10);
  const uint32_t hxl = h46 & l16;
  const uint32_t pr = A & ~h01 & ~(h2 & ~nz) & ~(h7 & lF);         // [!-~]
  const uint32_t dash = h2 & lD, dot = h2 & lE;
  out[BNL] = ~pr | al;                       // outside noLetters' class (templatize.go:14)
  out[BHX] = ~(dg | hxl);                    // outside [0-9A-Fa-f]
  out[DG] = dg;
  out[AT] = h4 & ~nz;
  out[HI] = b[7];
  out[DASH] = dash;
  out[SL] = h2 & lF;
  out[QM] = h3 & lF;
  const uint32_t bdom = ~(al | dg | dot | dash);   // outside [A-Za-z0-9.-] (emailRegex domain)
  out[BDOM] = bdom;
  out[BLOC] = bdom & ~((h5 & lF) | (h2 & l5B));    // outside [A-Za-z0-9._%+-] (emailRegex local part)
  out[DOT] = dot;
  out[NAL] = ~al;
}

// the 8 bit planes of one 32-byte row (x[d] = bytes 4d..4d+3)
OSE_UC void row_planes(const uint32_t* x, uint32_t* b) {
  uint32_t X[8];
  for (int d = 0; d < 8; d++) X[d] = x[d];
  for (int j = 0; j < 4; j++) xpose8(X[2 * j], X[2 * j + 1]);   // block j: bytes 8j..8j+7
  xpose4(X[0], X[2], X[4], X[6], b);       // planes 0-3: byte j from block j
  xpose4(X[1], X[3], X[5], X[7], b + 4);   // planes 4-7
}

// the class words of one 32-byte row
OSE_UC void row_classes(const uint32_t* x, uint32_t* out) {
  uint32_t b[8];
  row_planes(x, b);
  derive_planes(b, out);
}

}  // namespace uc
}  // namespace ose
