// attr_kernel.hip — the per-span condition of odigossampling's span_attribute
// rule on the GPU (internal/sampling/spanattribute.go:126-230, string /
// number / boolean conditions).  One lane per span: for every rule whose
// service is the span's resource service (AsString(service.name) ==
// ServiceName, spanattribute.go:130-132) it reads the span's value of the
// rule's attribute key from the key-major attr_type / attr_val columns and
// sets the rule's bit when the condition holds.  The bits of the rules the
// shim evaluates ("json" conditions) come in through host_bits.
//
// The kernel is HBM-bound on its columns for the common rule shapes (1 B
// type + 8 B value per span and key, 8 B of bits out); string conditions add
// the attribute's bytes, read through 16-byte vector loads from the arena.
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "devcfg.hpp"
#include "kernels.hpp"

namespace ose {

namespace {
constexpr int kAThreads = 256;

// strings.Contains(s[0:n], e[0:m]): m == 0 is true
__device__ bool contains(ByteReader& rd, uint32_t s, uint32_t n, const uint8_t* e, uint32_t m) {
  if (m == 0) return true;
  if (m > n) return false;
  const uint32_t first = e[0];
  for (uint32_t i = 0; i + m <= n; i++) {
    if (rd.at(s + i) != first) continue;
    uint32_t k = 1;
    while (k < m && rd.at(s + i + k) == e[k]) k++;
    if (k == m) return true;
  }
  return false;
}

__device__ bool equals(ByteReader& rd, uint32_t s, uint32_t n, const uint8_t* e, uint32_t m) {
  if (n != m) return false;
  for (uint32_t k = 0; k < n; k++)
    if (rd.at(s + k) != e[k]) return false;
  return true;
}

__device__ bool eval_rule(const AttrRuleDev& r, const uint8_t* blob, uint32_t t, uint64_t v, const uint8_t* arena) {
  switch (r.cond) {
    case kAttrCondStr: {
      // "exists": a non-empty string (spanattribute.go:137-141); every other
      // operation needs a string (:142-144)
      if (t != OSE_ATTR_STR) return false;
      const uint32_t off = (uint32_t)v, len = (uint32_t)(v >> 32);
      if (r.op == kAttrOpExists) return len != 0;
      ByteReader rd(arena);
      const uint8_t* e = blob + r.exp_off;
      switch (r.op) {
        case kAttrOpEq: return equals(rd, off, len, e, r.exp_len);
        case kAttrOpNe: return !equals(rd, off, len, e, r.exp_len);
        case kAttrOpContains: return contains(rd, off, len, e, r.exp_len);
        case kAttrOpNotContains: return !contains(rd, off, len, e, r.exp_len);
        case kAttrOpRegex: return r.dfa_off != 0 && dfa_match(blob, r.dfa_off, rd, off, off + len);
        default: return false;
      }
    }
    case kAttrCondNum: {
      const bool num = t == OSE_ATTR_INT || t == OSE_ATTR_DOUBLE;
      if (r.op == kAttrOpExists) return num;   // :180-184
      if (!r.num_ok || !num) return false;     // ParseFloat error / other types: continue
      const double x = t == OSE_ATTR_INT ? (double)(int64_t)v : __longlong_as_double((long long)v);
      switch (r.op) {
        case kAttrOpEq: return x == r.num;
        case kAttrOpNe: return x != r.num;
        case kAttrOpGt: return x > r.num;
        case kAttrOpLt: return x < r.num;
        case kAttrOpGe: return x >= r.num;
        case kAttrOpLe: return x <= r.num;
        default: return false;
      }
    }
    case kAttrCondBool:
      if (r.op == kAttrOpExists) return t == OSE_ATTR_BOOL;   // :223-227
      if (!r.bool_ok || t != OSE_ATTR_BOOL) return false;
      return r.op == kAttrOpEq && (v != 0) == (r.bool_val != 0);
    default:
      return false;
  }
}
}  // namespace

__global__ __launch_bounds__(kAThreads) void attr_eval_kernel(AttrArgs a) {
  const AttrCfgDev* h = reinterpret_cast<const AttrCfgDev*>(a.cfg);
  const AttrRuleDev* rules = reinterpret_cast<const AttrRuleDev*>(a.cfg + h->rules_off);
  const uint32_t nr = h->n_rules;
  const uint64_t stride = (uint64_t)gridDim.x * kAThreads;
  for (uint64_t i = (uint64_t)blockIdx.x * kAThreads + threadIdx.x; i < a.n_spans; i += stride) {
    const uint32_t svc = a.res_svc[a.resource[i]];
    // word w holds the bits of rules 64w..64w+63; the device rules are in
    // level order (increasing bit), so word w's are a contiguous stretch
    uint32_t k = 0;
    for (uint32_t w = 0; w < a.words; w++) {
      uint64_t bits = a.host_bits ? (a.host_bits[(uint64_t)w * a.n_spans + i] & a.host_mask[w]) : 0;
      for (; k < nr && rules[k].bit < 64 * (w + 1); k++) {
        const AttrRuleDev& r = rules[k];
        if (svc != r.svc) continue;
        const uint64_t j = (uint64_t)r.key * a.n_spans + i;
        const uint32_t t = a.type[j];
        if (t == OSE_ATTR_ABSENT) continue;   // Get(key) not found (:136-138)
        if (eval_rule(r, a.cfg, t, a.val[j], a.arena)) bits |= 1ull << (r.bit % 64);
      }
      a.out[(uint64_t)w * a.n_spans + i] = bits;
    }
  }
}

void launch_attr_eval(const AttrArgs& a, hipStream_t st) {
  const uint64_t blocks = std::min<uint64_t>((a.n_spans + kAThreads - 1) / kAThreads, 4096);
  if (blocks) hipLaunchKernelGGL(attr_eval_kernel, dim3((uint32_t)blocks), dim3(kAThreads), 0, st, a);
}

}  // namespace ose
