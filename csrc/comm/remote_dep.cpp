// Remote dependency engine (single-rank fallback until the shm/RCCL engine is
// attached by comm_init; see comm/shm_engine.cpp).
#include "comm.hpp"

namespace parsec {

static CommEngine* g_ce = nullptr;

CommEngine* comm_engine() { return g_ce; }
int comm_rank() { return g_ce ? g_ce->rank : 0; }
int comm_size() { return g_ce ? g_ce->size : 1; }
uint32_t comm_allreduce_max_u32(uint32_t v) { return g_ce ? (uint32_t)g_ce->allreduce_max(v) : v; }
int comm_barrier() { return g_ce ? g_ce->sync() : 0; }

void remote_dep_init(Context* ctx) {
  ctx->my_rank = comm_rank();
  ctx->nb_nodes = comm_size();
  set_debug_rank(ctx->my_rank);
}
void remote_dep_fini(Context* ctx) { (void)ctx; }
void remote_dep_on(Context* ctx) { (void)ctx; }
void remote_dep_off(Context* ctx) { (void)ctx; }
void remote_dep_progress_inline(Context* ctx) { (void)ctx; if (g_ce) g_ce->progress(); }
void remote_dep_new_taskpool(Context* ctx, Taskpool* tp) { (void)ctx; (void)tp; }
int remote_dep_activate(ExecutionStream* es, Taskpool* tp, RemoteDepsMsg& msg) {
  (void)es; (void)tp; (void)msg;
  fatal("remote activation requested but no communication engine is attached");
}
int comm_init(int rank, int size, const std::string& job_id, int gpu_ordinal) {
  (void)rank; (void)size; (void)job_id; (void)gpu_ordinal;
  return size == 1 ? 0 : -1;
}
void comm_fini() {}
TermdetModule* fourcounter_module() { return termdet_open_module("local"); }
void termdet_user_trigger_broadcast(Taskpool* tp) { (void)tp; }

}  // namespace parsec
