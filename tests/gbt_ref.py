"""Test infrastructure: groupbytrace restated over OTLP/JSON dicts (SURVEY.md
§8f-2).  The processor is opentelemetry-collector-contrib's
groupbytraceprocessor v0.141.0 (`collector/builder-config.yaml:73`), which is
not in the reference tree: parity is unpinned beyond its published
behaviour, restated here independently of the engine:

* ConsumeTraces splits the batch with batchpersignal.SplitTraces: for each
  ResourceSpans, for each ScopeSpans, one piece per trace id in order of
  first appearance (a copy of the resource and schema URL, one ScopeSpans
  with a copy of the scope and its schema URL, the trace's spans in order);
* each piece goes to the event machine in that order: an id already in the
  ring buffer gets the piece appended; otherwise the id takes the next ring
  slot (evicting — dropping — the trace there) and a timer of wait_duration
  is armed;
* when the timer fires the trace leaves the buffer and goes downstream as
  one ptrace.Traces of its pieces in arrival order;
* num_workers W > 1: the event machine hands a trace's events to worker
  workerIndexForTraceID(id) = FNV-1 64 of the 16 id bytes mod W, each worker
  with its own ring buffer of num_traces // W ids (eventMachineWorker.buffer).
  Traces released together come out in arming order here (Go's workers
  release them concurrently).

Releases happen at the caller's clock (`release(now)` fires every timer
with deadline <= now, in arming order).  A trace whose deadline has passed
takes no more spans even before that call: `consume(td, now)` treats its
id as unknown (a new trace), as contrib's timer would already have sent it.
A trace evicted after its deadline but before the release call is dropped
(the engine applies eviction per add).  One deliberate difference from
the Go code, which the engine shares: a timer releases the trace instance
it was armed for, so a trace evicted and created again is not released by
the old instance's timer.
"""
from __future__ import annotations

import copy


def split_traces(td: dict) -> list:
    """[(trace_id, ResourceSpans piece)] in SplitTraces order."""
    out = []
    for rs in td.get("resourceSpans") or []:
        for ss in rs.get("scopeSpans") or []:
            pieces = {}
            order = []
            for sp in ss.get("spans") or []:
                tid = (sp.get("traceId") or "").lower()
                if tid not in pieces:
                    piece = {"resource": copy.deepcopy(rs.get("resource") or {}),
                             "scopeSpans": [{"scope": copy.deepcopy(ss.get("scope") or {}), "spans": []}]}
                    if rs.get("schemaUrl"):
                        piece["schemaUrl"] = rs["schemaUrl"]
                    if ss.get("schemaUrl"):
                        piece["scopeSpans"][0]["schemaUrl"] = ss["schemaUrl"]
                    pieces[tid] = piece
                    order.append(tid)
                pieces[tid]["scopeSpans"][0]["spans"].append(copy.deepcopy(sp))
            out += [(t, pieces[t]) for t in order]
    return out


def _norm(tid: str) -> str:
    t = (tid or "").lower()
    return "" if t == "0" * 32 else t


def fnv1_64(data: bytes) -> int:
    """hash/fnv New64 (FNV-1: multiply, then xor)"""
    h = 0xCBF29CE484222325
    for b in data:
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
        h ^= b
    return h


def worker_index(tid: str, num_workers: int) -> int:
    return fnv1_64(bytes.fromhex(tid) if tid else bytes(16)) % num_workers


class GroupByTraceRef:
    def __init__(self, wait_ns: int, num_traces: int = 1_000_000, num_workers: int = 1):
        self.wait = wait_ns
        self.workers = num_workers
        self.size = num_traces // num_workers
        self.rings = [[None] * self.size for _ in range(num_workers)]   # instance ids
        self.index = [-1] * num_workers
        self.live = {}                    # trace id -> instance
        self.inst = {}                    # instance -> {"tid", "pieces", "deadline"}
        self.next = 0
        self.timers = []                  # (deadline, instance) in arming order
        self.evicted = 0

    def _expire(self, now: int) -> None:
        """Timers with deadline <= now have fired: their traces no longer take
        spans (a later span of the id starts a new trace), though they leave
        at the next release(now) call."""
        for d, k in self.timers:
            if d > now:
                break
            t = self.inst.get(k)
            if t is not None and self.live.get(t["tid"]) == k:
                del self.live[t["tid"]]

    def consume(self, td: dict, now: int) -> None:
        self._expire(now)
        for tid, piece in split_traces(td):
            tid = _norm(tid)
            if tid in self.live:
                self.inst[self.live[tid]]["pieces"].append(piece)
                continue
            w = worker_index(tid, self.workers)
            self.index[w] = (self.index[w] + 1) % self.size
            ring = self.rings[w]
            old = ring[self.index[w]]
            if old is not None and old in self.inst:   # evicted: dropped
                if self.live.get(self.inst[old]["tid"]) == old:
                    del self.live[self.inst[old]["tid"]]
                del self.inst[old]
                self.evicted += 1
            k = self.next
            self.next += 1
            ring[self.index[w]] = k
            self.live[tid] = k
            self.inst[k] = {"tid": tid, "pieces": [piece]}
            self.timers.append((now + self.wait, k))

    def release(self, now: int) -> list:
        """The traces whose timers fired: [[piece, ...], ...] in firing order."""
        fired = [k for d, k in self.timers if d <= now]
        self.timers = [(d, k) for d, k in self.timers if d > now]
        out = []
        for k in fired:
            t = self.inst.pop(k, None)
            if t is None:
                continue   # evicted earlier
            if self.live.get(t["tid"]) == k:   # (an expired trace has left `live` already)
                del self.live[t["tid"]]
            out.append(t["pieces"])
        return out
