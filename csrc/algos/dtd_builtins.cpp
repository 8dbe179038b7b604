// Built-in GPU bodies usable as DTD chores from any front-end (C++, C, Python):
// the body reads its sizes from the task's VALUE arguments and its device
// pointers from the engine, and enqueues into the round's kernel batch.
//   "dgemm"  : A(IN) B(IN) C(INOUT) | m n k (int32) alpha beta (double) [transB int32, default 1]
//   "dsyrk"  : A(IN) C(INOUT)       | n k (int32) alpha beta (double)   (lower, C += alpha A A^T)
//   "dtrsm"  : L(IN) B(INOUT)       | m n (int32)                        (B := B L^-T)
//   "dpotrf" : A(INOUT)             | n (int32)
//   "memset" : A(OUTPUT)            | bytes (int64) value (int32)
#include <hip/hip_runtime_api.h>

#include "../device/device.hpp"
#include "../dtd/dtd.hpp"

namespace parsec {

namespace {
struct Vals {
  std::vector<const void*> v;
  explicit Vals(Task* t) {
    auto* d = static_cast<dtd::DtdTask*>(t);
    for (auto& a : d->args)
      if ((a.op & dtd::OP_MASK) == dtd::VALUE) v.push_back(a.ptr);
  }
  int32_t i(size_t k, int32_t dflt = 0) const { return k < v.size() ? *static_cast<const int32_t*>(v[k]) : dflt; }
  int64_t l(size_t k, int64_t dflt = 0) const { return k < v.size() ? *static_cast<const int64_t*>(v[k]) : dflt; }
  double d(size_t k, double dflt = 0) const { return k < v.size() ? *static_cast<const double*>(v[k]) : dflt; }
};
double* dptr(GpuExecContext* c, Task* t, int argi) {
  int f = dtd::task_arg_flow(t, argi);
  return f >= 0 ? static_cast<double*>(c->ptr(f)) : nullptr;
}
int argidx_of_flow(Task* t, int flow) {
  auto* d = static_cast<dtd::DtdTask*>(t);
  for (size_t i = 0; i < d->args.size(); ++i) if (d->args[i].flow == flow) return (int)i;
  return -1;
}
}  // namespace

std::function<int(GpuExecContext*, Task*)> builtin_dtd_gpu_body(const std::string& name) {
  if (name == "dgemm")
    return [](GpuExecContext* c, Task* t) {
      Vals v(t);
      GemmDesc g{};
      g.A = dptr(c, t, argidx_of_flow(t, 0)); g.B = dptr(c, t, argidx_of_flow(t, 1)); g.C = dptr(c, t, argidx_of_flow(t, 2));
      g.m = v.i(0); g.n = v.i(1); g.k = v.i(2);
      g.alpha = v.d(3, 1.0); g.beta = v.d(4, 1.0);
      g.transA = 0; g.transB = (uint8_t)v.i(5, 1); g.lower_only = 0; g.a_lower = 0;
      g.lda = g.m; g.ldb = g.transB ? g.n : g.k; g.ldc = g.m;
      c->batch->gemm.push_back(g);
      return (int)HOOK_DONE;
    };
  if (name == "dsyrk")
    return [](GpuExecContext* c, Task* t) {
      Vals v(t);
      GemmDesc g{};
      g.A = dptr(c, t, argidx_of_flow(t, 0)); g.B = g.A; g.C = dptr(c, t, argidx_of_flow(t, 1));
      g.m = g.n = v.i(0); g.k = v.i(1);
      g.alpha = v.d(2, -1.0); g.beta = v.d(3, 1.0);
      g.transA = 0; g.transB = 1; g.lower_only = 1; g.a_lower = 0;
      g.lda = g.ldb = g.ldc = g.m;
      c->batch->gemm.push_back(g);
      return (int)HOOK_DONE;
    };
  if (name == "dtrsm")
    return [](GpuExecContext* c, Task* t) {
      Vals v(t);
      TrsmDesc d;
      d.L = dptr(c, t, argidx_of_flow(t, 0)); d.B = dptr(c, t, argidx_of_flow(t, 1));
      d.m = v.i(0); d.n = v.i(1); d.ldl = d.n; d.ldb = d.m; d.trans = 1;
      c->batch->trsm.push_back(d);
      return (int)HOOK_DONE;
    };
  if (name == "dpotrf")
    return [](GpuExecContext* c, Task* t) {
      Vals v(t);
      int n = v.i(0);
      c->batch->potrf.push_back(PotrfDesc{dptr(c, t, argidx_of_flow(t, 0)), n, n, nullptr});
      return (int)HOOK_DONE;
    };
  if (name == "memset")
    return [](GpuExecContext* c, Task* t) {
      Vals v(t);
      void* p = c->ptr(0);
      size_t bytes = (size_t)v.l(0);
      int val = v.i(1);
      c->batch->generic.push_back([p, bytes, val](hipStream_t s) { (void)hipMemsetAsync(p, val, bytes, s); });
      return (int)HOOK_DONE;
    };
  fatal("unknown built-in DTD GPU body '%s'", name.c_str());
}

}  // namespace parsec
