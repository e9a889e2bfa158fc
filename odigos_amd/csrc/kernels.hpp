// kernels.hpp — host-side launch interfaces of the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/odigos_amd.h"

namespace ose {

struct UrlKernelArgs {
  uint64_t n_spans;
  uint32_t n_tiles;
  const uint8_t* arena;
  const uint8_t* url_flags;
  const uint8_t* kind;
  const uint32_t* resource;
  const uint8_t* res_url_ok;   // may be null (no include/exclude)
  const ose_strref* path;
  uint8_t* url_out;
  ose_strref* tmpl;
  uint8_t* out_arena;
  uint64_t out_cap;
  const uint8_t* cfg;          // UrlCfgDev blob
  uint32_t* tile_counter;      // zeroed before launch
  uint64_t* tile_status;       // [n_tiles], zeroed before launch
  uint32_t* error;             // bit0 look-back timeout, bit1 output overflow
  uint64_t* used;              // bytes written (optional)
};
constexpr uint32_t kUrlTile = 1024;   // spans per workgroup tile (url_kernel.hip kTile)
void launch_url_template(const UrlKernelArgs& a, hipStream_t st);

}  // namespace ose
