#include "recursive.hpp"

namespace parsec {

int recursive_call(ExecutionStream* es, Task* parent, Taskpool* inner, std::function<void(Taskpool*)> on_done) {
  Context* ctx = parent->taskpool->context;
  if (!ctx) fatal("recursive_call: the parent taskpool is not attached to a context");
  auto prev = inner->on_complete;
  inner->on_complete = [ctx, parent, prev, on_done](Taskpool* tp) {
    if (prev) prev(tp);
    if (on_done) on_done(tp);
    ExecutionStream* cur = my_execution_stream();
    ExecutionStream* e = cur && cur->ctx == ctx ? cur : ctx->all_es[0];
    complete_task_execution(e, parent);
    return 0;
  };
  (void)es;
  context_add_taskpool(ctx, inner);
  return HOOK_ASYNC;
}

}  // namespace parsec
