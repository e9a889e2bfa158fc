// pb_device.hpp — protobuf wire-format reading on the device, shared by the
// OTLP decoder (otlp_kernel.hip) and the re-encoder (encode_kernel.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/odigos_amd.h"
#include "device_common.hpp"

#ifndef OSE_PB_NO_FORCE
#define OSE_PB_INL __forceinline__
#define OSE_PB_LOOP _Pragma("nounroll")
#else
#define OSE_PB_INL
#define OSE_PB_LOOP
#endif

namespace ose {
namespace pbdev {

__device__ __forceinline__ uint32_t sov(uint64_t x) { return (uint32_t)((64 - __clzll(x | 1) + 6) / 7); }
__device__ __forceinline__ uint64_t field_len(uint64_t l) { return 1 + sov(l) + l; }
__device__ __forceinline__ uint64_t str_field(uint64_t l) { return l ? field_len(l) : 0; }
__device__ OSE_PB_INL uint64_t varint_field(uint64_t v) { return v ? 1 + sov(v) : 0; }

struct Rd {
  ByteReader br;
  uint32_t i, end;
  bool bad;
  __device__ Rd(const uint8_t* base, uint32_t s, uint32_t e) : br(base), i(s), end(e), bad(false) {}
  __device__ __forceinline__ bool more() const { return !bad && i < end; }
  __device__ OSE_PB_INL uint64_t varint() {
    uint64_t v = 0;
    OSE_PB_LOOP
    for (uint32_t s = 0; s < 64; s += 7) {
      if (i >= end) break;
      const uint32_t b = br.at(i++);
      v |= (uint64_t)(b & 0x7F) << s;
      if (b < 0x80) return v;
    }
    bad = true;
    return 0;
  }
  __device__ OSE_PB_INL uint64_t fixed(uint32_t nb) {
    if (i + nb > end) { bad = true; return 0; }
    uint64_t v = 0;
    OSE_PB_LOOP
    for (uint32_t k = 0; k < nb; k++) v |= (uint64_t)br.at(i + k) << (8 * k);
    i += nb;
    return v;
  }
  // LEN payload [s, s + l)
  __device__ OSE_PB_INL bool len(uint32_t& s, uint32_t& l) {
    const uint64_t x = varint();
    if (bad || x > end - i) { bad = true; return false; }
    s = i;
    l = (uint32_t)x;
    i += l;
    return true;
  }
  // an unknown field (groups go to the host pass)
  __device__ OSE_PB_INL bool skip(uint32_t wt) {
    uint32_t s, l;
    switch (wt) {
      case 0: varint(); break;
      case 1: fixed(8); break;
      case 2: len(s, l); break;
      case 5: fixed(4); break;
      default: bad = true;
    }
    return !bad;
  }
  __device__ OSE_PB_INL bool tag(uint32_t& f, uint32_t& wt) {
    const uint64_t t = varint();
    f = (uint32_t)(t >> 3);
    wt = (uint32_t)(t & 7);
    if (bad || f == 0 || (t >> 3) > 0x1FFFFFFFull || wt == 3 || wt == 4) bad = true;
    return !bad;
  }
};

// a value of interest: AnyValue type (OSE_ATTR_* plus kNested / kAttrBytes) and payload
constexpr uint32_t kNested = 6, kAttrBytes = 7;
struct Val {
  uint32_t type;   // OSE_ATTR_ABSENT when the key was not seen
  uint32_t off, len;
  uint64_t v;
};

// AnyValue [s, e): the last oneof field wins; returns its pdata size
// contribution (ProtoSizer::any_value) or sets nested / bad
__device__ OSE_PB_INL uint64_t any_value(Rd& r, uint32_t s, uint32_t e, Val& out) {
  const uint32_t save_i = r.i, save_end = r.end;
  r.i = s;
  r.end = e;
  out.type = OSE_ATTR_OTHER;   // empty AnyValue: TEmpty (size 0)
  out.off = out.len = 0;
  out.v = 0;
  uint64_t sz = 0;
  uint32_t f, wt;
  while (r.more() && r.tag(f, wt)) {
    uint32_t ps, pl;
    switch (f) {
      case 1:
        if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
        out.type = OSE_ATTR_STR; out.off = ps; out.len = pl; out.v = 0;
        sz = field_len(pl);
        break;
      case 2:
        if (wt != 0) { r.bad = true; break; }
        out.v = r.varint() != 0; out.type = OSE_ATTR_BOOL;
        sz = 2;
        break;
      case 3:
        if (wt != 0) { r.bad = true; break; }
        out.v = r.varint(); out.type = OSE_ATTR_INT;
        sz = 1 + sov(out.v);
        break;
      case 4:
        if (wt != 1) { r.bad = true; break; }
        out.v = r.fixed(8); out.type = OSE_ATTR_DOUBLE;
        sz = 9;
        break;
      case 5:
      case 6:
        if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
        out.type = kNested;
        break;
      case 7:
        if (wt != 2 || !r.len(ps, pl)) { r.bad = true; break; }
        out.type = kAttrBytes; out.off = ps; out.len = pl;
        sz = field_len(pl);
        break;
      default:
        r.skip(wt);
    }
  }
  if (out.type == OSE_ATTR_OTHER) sz = 0;
  r.i = save_i;
  r.end = save_end;
  return sz;
}

}  // namespace pbdev
}  // namespace ose
