// Recursive tasks: a task body runs an inner taskpool and its successors are
// released only when that taskpool terminates (reference recursive.h:20-76,
// parsec_recursivecall). Typical use, inside a CPU or DEV_RECURSIVE chore:
//
//     auto* inner = build_inner_taskpool(...);
//     return parsec::recursive_call(es, this_task, inner);   // == HOOK_ASYNC
//
// The inner taskpool is added to the parent's context; on termination the
// optional callback runs, then the parent task completes. The caller keeps
// ownership of `inner` (free it after its termination, e.g. in the callback's
// owner or after context_wait).
#pragma once
#include <functional>

#include "runtime.hpp"

namespace parsec {

int recursive_call(ExecutionStream* es, Task* parent, Taskpool* inner, std::function<void(Taskpool*)> on_done = nullptr);

}  // namespace parsec
