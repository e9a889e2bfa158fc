// Host check of blob.hpp's uint32 offset guard: a section that would carry
// the blob past 4 GiB is refused (overflow set, nothing appended) instead of
// wrapping the offsets the device tables hold.  Run by test_abi.py.
#include <cstdio>

#include "../odigos_amd/csrc/blob.hpp"

int main() {
  using ose::Blob;
  Blob bl;
  uint32_t a = 7;
  uint32_t off = bl.put(&a, 1);
  if (off != 0 || bl.overflow || bl.b.size() != 4) { std::puts("small put"); return 1; }
  // 5 GiB of uint8 from a null pointer: the guard must refuse it before any read
  const uint8_t* none = nullptr;
  bl.put(none, (size_t)5 << 30);
  if (!bl.overflow || bl.b.size() > 64) { std::puts("huge put not refused"); return 1; }
  // later puts stay refused
  if (bl.put(&a, 1) != 0 || bl.b.size() > 64) { std::puts("put after overflow"); return 1; }
  // the edge: one put that ends exactly at kMaxBytes is fine in arithmetic,
  // one byte more is not (checked without allocating)
  Blob e;
  if ((uint64_t)e.b.size() + Blob::kMaxBytes > Blob::kMaxBytes) { std::puts("edge"); return 1; }
  e.put(none, (size_t)Blob::kMaxBytes + 1);
  if (!e.overflow || !e.b.empty()) { std::puts("edge +1 not refused"); return 1; }
  std::puts("OK");
  return 0;
}
