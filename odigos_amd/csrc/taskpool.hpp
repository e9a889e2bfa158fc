// taskpool.hpp — a process-wide pool of host worker threads for the
// per-batch parallel loops (the OTLP structural walk, the re-encoder): a
// gateway calls once per batch, and at the batch processor's 8192 spans
// spawning threads per call costs as much as the work.
#pragma once
#include <functional>

namespace ose {

// Runs fn(0) .. fn(n-1), fn(0) on the calling thread, the rest on the pool
// (the caller helps with queued tasks while it waits, so nested or
// concurrent callers cannot starve).  Returns when all have finished.
void parallel_run(int n, const std::function<void(int)>& fn);

// Worker threads available (the pool's size + the caller).
int parallel_width();

}  // namespace ose
