// Small builders for hand-written PTG task classes (what parsec-ptgpp emits
// for .jdf sources, written directly in C++ for the built-in algorithms).
#pragma once
#include <string>
#include <vector>

#include "../data/collections.hpp"
#include "../ptg/ptg.hpp"

namespace parsec {
namespace algos {
namespace ir {

using namespace ptg;

inline LocalDef range_local(const std::string& n, Expr lo, Expr hi) {
  LocalDef l;
  l.name = n; l.is_range = true; l.is_param = true; l.lo = std::move(lo); l.hi = std::move(hi);
  return l;
}
inline Expr cst(int64_t v) { return [v](const Taskpool*, const int32_t*) { return v; }; }
inline Expr loc(int i) { return [i](const Taskpool*, const int32_t* L) { return (int64_t)L[i]; }; }
inline Expr locp(int i, int64_t d) { return [i, d](const Taskpool*, const int32_t* L) { return (int64_t)L[i] + d; }; }
inline CallArg val(Expr e) { CallArg a; a.value = std::move(e); return a; }
inline CallArg rng(Expr lo, Expr hi) { CallArg a; a.is_range = true; a.lo = std::move(lo); a.hi = std::move(hi); return a; }
inline DepTarget task(const std::string& tc, const std::string& flow, std::vector<CallArg> args) {
  DepTarget t; t.kind = DEP_TASK; t.tc_name = tc; t.flow_name = flow; t.args = std::move(args); return t;
}
inline DepTarget data(DataCollection* A, Expr m, Expr n) {
  DepTarget t; t.kind = DEP_DATA; t.dc = [A](const Taskpool*) { return A; }; t.args = {val(std::move(m)), val(std::move(n))}; return t;
}
inline DepTarget data1(DataCollection* A, Expr m) {
  DepTarget t; t.kind = DEP_DATA; t.dc = [A](const Taskpool*) { return A; }; t.args = {val(std::move(m))}; return t;
}
inline DepTarget newbuf(int adt_index) { DepTarget t; t.kind = DEP_NEW; t.datatype_index = adt_index; return t; }
inline Dep always(DepTarget t) { Dep d; d.then_t = std::move(t); return d; }
inline Dep cond(Guard g, DepTarget a, DepTarget b) { Dep d; d.guard = std::move(g); d.then_t = std::move(a); d.has_else = true; d.else_t = std::move(b); return d; }
inline Dep when(Guard g, DepTarget a) { Dep d; d.guard = std::move(g); d.then_t = std::move(a); return d; }
inline double* fptr(Task* t, int f) {
  DataCopy* c = t->data[f].data_out ? t->data[f].data_out : t->data[f].data_in;
  return c ? static_cast<double*>(c->device_private) : nullptr;
}

}  // namespace ir
}  // namespace algos
}  // namespace parsec
