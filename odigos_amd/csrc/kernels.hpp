// kernels.hpp — host-side launch interfaces of the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/odigos_amd.h"

namespace ose {

// odigosurltemplate: three launches on one stream (url_kernel.hip).
//   url_plan_kernel  one wave per 64-span group: plan + output length per span
//   url_scan_kernel  exclusive scan of the per-group output sums
//   url_emit_kernel  one wave per group: template bytes + refs
struct UrlKernelArgs {
  uint64_t n_spans;
  uint32_t n_groups;           // ceil(n_spans / kUrlGroup)
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
  // workspace
  uint32_t* plan_len;          // [n_spans] output length
  uint32_t* plan_meta;         // [n_spans] mode/lead/slow/url_out/field
  uint64_t* plan_code;         // [n_spans] per-segment name ids
  uint64_t* group_sum;         // [n_groups]
  uint64_t* group_base;        // [n_groups] exclusive prefix
  uint32_t n_scan_tiles;       // ceil(n_groups / kUrlScanTile)
  uint32_t* scan_counter;      // zeroed before launch
  uint64_t* scan_status;       // [n_scan_tiles], zeroed before launch
  uint32_t* error;             // bit0 look-back timeout, bit1 output overflow
  uint64_t* used;              // bytes written (optional)
  uint32_t ablate;             // diagnostics only (OSE_URL_ABLATE): 1 skip emission, 2 skip planning, 4 skip bitmaps
  uint64_t* dbg;               // diagnostics only (ablate & 512): per-section clock sums
};
constexpr uint32_t kUrlGroup = 64;       // spans per wave group (url_kernel.hip kWave)
constexpr uint32_t kUrlScanTile = 1024;  // groups per scan workgroup (url_kernel.hip kScanThreads)
// workspace bytes the URL stage needs for n spans (engine.cpp run_url layout)
inline size_t url_workspace_bytes(uint64_t n) {
  const uint64_t g = (n + kUrlGroup - 1) / kUrlGroup;
  const uint64_t t = (g + kUrlScanTile - 1) / kUrlScanTile;
  return 256 + n * 16 + g * 16 + t * 8 + 1024;
}
void launch_url_plan(const UrlKernelArgs& a, hipStream_t st);
void launch_url_scan(const UrlKernelArgs& a, hipStream_t st);
void launch_url_emit(const UrlKernelArgs& a, hipStream_t st);

}  // namespace ose
