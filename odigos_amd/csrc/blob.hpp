// blob.hpp — builder of the read-only device tables (devcfg.hpp): 16-byte
// aligned sections appended to one byte vector, uploaded once per engine.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

#include "devcfg.hpp"
#include "regex_dfa.hpp"

namespace ose {

// Section offsets (and DfaDev's trans_off / acc_off) are uint32: a blob
// that would pass kMaxBytes appends nothing more and sets `overflow`, which
// the table builders turn into OSE_ENOTSUP (sixteen 256 MiB DFAs would
// otherwise wrap the offsets and point the kernels at the wrong tables).
struct Blob {
  static constexpr uint64_t kMaxBytes = 0xFFFFFFFFull - 64;
  std::vector<uint8_t> b;
  bool overflow = false;
  uint32_t align() {
    while (b.size() % 16) b.push_back(0);
    if (b.size() > kMaxBytes) overflow = true;
    return overflow ? 0u : (uint32_t)b.size();
  }
  template <typename T>
  uint32_t put(const T* p, size_t n) {
    uint32_t off = align();
    if (overflow || (uint64_t)b.size() + (uint64_t)n * sizeof(T) > kMaxBytes) {
      overflow = true;
      return 0;
    }
    const uint8_t* s = reinterpret_cast<const uint8_t*>(p);
    b.insert(b.end(), s, s + n * sizeof(T));
    return off;
  }
  template <typename T>
  T* at(uint32_t off) { return reinterpret_cast<T*>(b.data() + off); }
};

inline uint32_t put_dfa(Blob& bl, const Dfa& d) {
  DfaDev h{};
  h.nclasses = d.nclasses;
  h.nstates = d.nstates;
  h.start = d.start;
  h.match = d.match;
  h.hi_n = (uint32_t)d.hi_lo.size();
  std::memcpy(h.ascii, d.ascii_class, 128);
  h.wide = d.nstates > 65535 ? 1u : 0u;
  uint32_t off = bl.put(&h, 1);
  std::vector<uint32_t> hr;
  for (size_t k = 0; k < d.hi_lo.size(); k++) { hr.push_back(d.hi_lo[k]); hr.push_back(d.hi_hi[k]); hr.push_back(d.hi_cls[k]); }
  uint32_t hoff = bl.put(hr.data(), hr.size());
  h.wide = d.nstates > 65535 ? 1u : 0u;
  uint32_t toff;
  if (h.wide) {
    toff = bl.put(d.trans.data(), d.trans.size());
  } else {
    std::vector<uint16_t> t16(d.trans.begin(), d.trans.end());
    toff = bl.put(t16.data(), t16.size());
  }
  uint32_t aoff = bl.put(d.accept_end.data(), d.accept_end.size());
  if (bl.overflow) return 0;
  DfaDev* hp = bl.at<DfaDev>(off);
  hp->hi_off = hoff;
  hp->trans_off = toff;
  hp->acc_off = aoff;
  return off;
}


}  // namespace ose
