// sampling_host.cpp — odigossampling rule tables (built once per engine).
#include <algorithm>

#include "engine_internal.hpp"
#include "kernels.hpp"
#include "host.hpp"

namespace ose {

// Interns every service name a rule compares against (latency.go:55,
// servicename.go:40, spanattribute.go:130); the shim maps resources onto
// these ids with ose_engine_service_id.
int Engine::build_sampling_tables() {
  service_ids.clear();
  if (!has_sampling) return 0;
  for (auto& kv : intern_services(sampling)) service_ids.emplace(kv.first, kv.second);
  return 0;
}

size_t Engine::workspace_bytes(uint64_t n_spans) const {
  return url_workspace_bytes(n_spans);
}

}  // namespace ose
