// Python bindings (pybind11) for the parsec-amd runtime.
// Blocking calls release the GIL; Python task bodies re-acquire it on the
// worker thread that runs them.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "../algos/linalg.hpp"
#include "../algos/stencil3d.hpp"
#include "../core/recursive.hpp"
#include "../comm/comm.hpp"
#include "../core/runtime.hpp"
#include "../data/collections.hpp"
#include "../device/device.hpp"
#include "../device/hip_device.hpp"
#include "../dtd/dtd.hpp"
#include "../prof/profiling.hpp"
#include "../ptg/ptg.hpp"

namespace py = pybind11;
using namespace parsec;

extern "C" int parsec_amd_dgemm_batch(const GemmDesc* descs, int n, void* stream);
extern "C" int parsec_amd_gemm_tile_policy(int p);
extern "C" int parsec_amd_gemm_splitk(int on);
extern "C" int parsec_amd_potrf_steps(int on);
extern "C" int parsec_amd_potrf_stamps(long long* out);
extern "C" int parsec_amd_dtrsm_batch(const TrsmDesc* descs, int n, void* stream);
extern "C" int parsec_amd_dpotrf_tile(double* A, int n, int lda, int* info, void* stream);
extern "C" int parsec_amd_trsm_w_batch(const parsec::TrsmGemmDesc* d, int n, void* stream);
extern "C" int parsec_amd_dpotrf_tile_w(double* A, int n, int lda, int* info, double* W, int ldw, void* stream, int pack);
extern "C" int parsec_amd_qr_panel(const parsec::QrPanelDesc* d, int n, void* stream);
extern "C" int parsec_amd_qr_profile(unsigned long long* out);
extern "C" int parsec_amd_qr_apply(const parsec::QrApplyDesc* d, int n, void* ws, void* stream);
extern "C" size_t parsec_amd_qr_apply_ws(const parsec::QrApplyDesc* d, int n);
namespace parsec { void register_builtin_dtd_gpu_bodies(); std::function<int(GpuExecContext*, Task*)> builtin_dtd_gpu_body(const std::string& name); }

namespace {

struct PxContext {
  Context* ctx = nullptr;
  std::vector<py::object> keep;  // python objects referenced by running taskpools
};

static py::dtype dtype_of(int mtype) {
  switch (mtype) {
    case MATRIX_BYTE: return py::dtype::of<uint8_t>();
    case MATRIX_INTEGER: return py::dtype::of<int32_t>();
    case MATRIX_FLOAT: return py::dtype::of<float>();
    case MATRIX_DOUBLE: return py::dtype::of<double>();
    case MATRIX_COMPLEX_FLOAT: return py::dtype("complex64");
    case MATRIX_COMPLEX_DOUBLE: return py::dtype("complex128");
  }
  return py::dtype::of<double>();
}

// numpy view of a host buffer laid out as an (mb x nb) column-major tile
static py::array tile_view(void* p, int mtype, int64_t mb, int64_t nb, size_t esz) {
  if (!p) return py::none();
  std::vector<py::ssize_t> shape{(py::ssize_t)mb, (py::ssize_t)nb};
  std::vector<py::ssize_t> strides{(py::ssize_t)esz, (py::ssize_t)(esz * mb)};
  return py::array(dtype_of(mtype), shape, strides, p, py::capsule(p, [](void*) {}));
}

struct PyTask {
  Task* t;
};

static py::object dtd_arg(Task* t, int i) {
  auto* dt = static_cast<dtd::DtdTask*>(t);
  if (i < 0 || i >= (int)dt->args.size()) throw py::index_error("argument index");
  const dtd::Arg& a = dt->args[i];
  int op = a.op & dtd::OP_MASK;
  if (a.flow >= 0) {
    DataCopy* c = t->data[a.flow].data_in;
    if (!c) return py::none();
    Data* d = c->original;
    if (c->device_index != 0) return py::int_((uintptr_t)c->device_private);
    // received remote copies carry a bare Data: type them through the tile's collection
    DataCollection* dcc = (d && d->dc) ? d->dc : (a.tile ? a.tile->dc : nullptr);
    if (dcc) {
      if (auto* st = dynamic_cast<SubTileMatrix*>(dcc)) {  // strided view: ld = the parent tile's
        const size_t es = st->elem_size;
        return py::array(py::dtype(st->mtype == MATRIX_INTEGER ? "int32" : (st->mtype == MATRIX_FLOAT ? "float32" : "float64")), {(py::ssize_t)st->mb, (py::ssize_t)st->nb},
                         {(py::ssize_t)es, (py::ssize_t)(es * st->plda)}, c->device_private, py::capsule(c->device_private, [](void*) {}));
      }
      if (auto* tm = dynamic_cast<TiledMatrix*>(dcc)) return tile_view(c->device_private, tm->mtype, tm->mb, tm->nb, tm->elem_size);
    }
    size_t n = d ? d->nb_elts : 0;
    return py::array(py::dtype::of<uint8_t>(), {(py::ssize_t)n}, {1}, c->device_private, py::capsule(c->device_private, [](void*) {}));
  }
  if (op == dtd::VALUE) return py::bytes(static_cast<const char*>(a.ptr), (size_t)a.size);
  if (op == dtd::SCRATCH) return py::array(py::dtype::of<uint8_t>(), {(py::ssize_t)a.size}, {1}, a.ptr, py::capsule(a.ptr, [](void*) {}));
  if (op == dtd::REF) return py::int_((uintptr_t)a.ptr);
  return py::none();
}

template <class M>
static void bind_tiled_common(py::class_<M, TiledMatrix>& c) { (void)c; }

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "parsec-amd native runtime";

  // ----------------------------------------------------------- constants
  m.attr("HOOK_DONE") = (int)HOOK_DONE;
  m.attr("HOOK_AGAIN") = (int)HOOK_AGAIN;
  m.attr("HOOK_NEXT") = (int)HOOK_NEXT;
  m.attr("HOOK_DISABLE") = (int)HOOK_DISABLE;
  m.attr("HOOK_ASYNC") = (int)HOOK_ASYNC;
  m.attr("HOOK_ERROR") = (int)HOOK_ERROR;
  m.attr("DEV_CPU") = (int)DEV_CPU;
  m.attr("DEV_RECURSIVE") = (int)DEV_RECURSIVE;
  m.attr("DEV_HIP") = (int)DEV_HIP;
  m.attr("DEV_TEMPLATE") = (int)DEV_TEMPLATE;
  m.attr("DEV_ALL") = (int)DEV_ALL;
  m.attr("INPUT") = (int)dtd::INPUT;
  m.attr("OUTPUT") = (int)dtd::OUTPUT;
  m.attr("INOUT") = (int)dtd::INOUT;
  m.attr("ATOMIC_WRITE") = (int)dtd::ATOMIC_WRITE;
  m.attr("SCRATCH") = (int)dtd::SCRATCH;
  m.attr("VALUE") = (int)dtd::VALUE;
  m.attr("REF") = (int)dtd::REF;
  m.attr("AFFINITY") = (int)dtd::AFFINITY;
  m.attr("DONT_TRACK") = (int)dtd::DONT_TRACK;
  m.attr("PUSHOUT") = (int)dtd::PUSHOUT;
  m.attr("PULLIN") = (int)dtd::PULLIN;
  m.attr("PASSED_BY_REF") = (int)dtd::PASSED_BY_REF;
  m.attr("MATRIX_BYTE") = (int)MATRIX_BYTE;
  m.attr("MATRIX_INTEGER") = (int)MATRIX_INTEGER;
  m.attr("MATRIX_FLOAT") = (int)MATRIX_FLOAT;
  m.attr("MATRIX_DOUBLE") = (int)MATRIX_DOUBLE;
  m.attr("MATRIX_COMPLEX_FLOAT") = (int)MATRIX_COMPLEX_FLOAT;
  m.attr("MATRIX_COMPLEX_DOUBLE") = (int)MATRIX_COMPLEX_DOUBLE;
  m.attr("MATRIX_FULL") = (int)MATRIX_FULL;
  m.attr("MATRIX_LOWER") = (int)MATRIX_LOWER;
  m.attr("MATRIX_UPPER") = (int)MATRIX_UPPER;

  // --------------------------------------------------------------- params
  m.def("mca_set", [](const std::string& n, const std::string& v) { ParamRegistry::instance().set_override(n, v); });
  m.def("mca_unset", [](const std::string& n) { ParamRegistry::instance().clear_override(n); });
  m.def("mca_get", [](const std::string& n) -> py::object {
    std::string v;
    if (ParamRegistry::instance().lookup(n, v)) return py::str(v);
    return py::none();
  });
  m.def("mca_dump", []() {
    py::list out;
    for (auto& p : ParamRegistry::instance().dump()) out.append(py::make_tuple(p.full_name, p.value, p.source, p.help));
    return out;
  });
  m.def("mca_parse_cmdline", [](std::vector<std::string> args) { return ParamRegistry::instance().parse_cmdline(args); });
  m.def("schedulers", []() {
    py::list out;
    for (auto& c : scheduler_components()) out.append(py::make_tuple(c.name, c.priority, c.description));
    return out;
  });
  m.def("termdet_modules", []() { return termdet_available(); });
  m.def("pins_modules", []() { return pins_modules_available(); });

  // -------------------------------------------------------------- context
  py::class_<PxContext>(m, "Context")
      .def(py::init([](int nb_cores, std::vector<std::string> args) {
             auto* pc = new PxContext();
             py::gil_scoped_release rel;
             pc->ctx = context_init(nb_cores, args);
             return pc;
           }),
           py::arg("nb_cores") = -1, py::arg("args") = std::vector<std::string>{})
      .def("add_taskpool", [](PxContext& c, py::object tpo) {
        Taskpool* tp = tpo.cast<Taskpool*>();
        c.keep.push_back(tpo);
        py::gil_scoped_release rel;
        return context_add_taskpool(c.ctx, tp);
      })
      .def("start", [](PxContext& c) { py::gil_scoped_release rel; return context_start(c.ctx); })
      .def("test", [](PxContext& c) { return context_test(c.ctx); })
      .def("wait", [](PxContext& c) {
        {
          py::gil_scoped_release rel;
          context_wait(c.ctx);
        }
        c.keep.clear();
        return 0;
      })
      .def("fini", [](PxContext& c) {
        if (!c.ctx) return 0;
        {
          py::gil_scoped_release rel;
          context_fini(&c.ctx);
        }
        c.keep.clear();
        return 0;
      })
      .def_property_readonly("nb_cores", [](PxContext& c) { return c.ctx->nb_cores; })
      .def_property_readonly("nb_vp", [](PxContext& c) { return c.ctx->nb_vp; })
      .def_property_readonly("rank", [](PxContext& c) { return c.ctx->my_rank; })
      .def_property_readonly("nb_nodes", [](PxContext& c) { return c.ctx->nb_nodes; })
      .def_property_readonly("scheduler", [](PxContext& c) { return c.ctx->scheduler_name; })
      .def_property_readonly("active_taskpools", [](PxContext& c) { return c.ctx->active_taskpools.load(); })
      .def_property_readonly("alive", [](PxContext& c) { return c.ctx != nullptr; });

  // ------------------------------------------------------------- taskpools
  py::class_<Taskpool>(m, "Taskpool")
      .def_property("name", [](Taskpool& t) { return t.taskpool_name; }, [](Taskpool& t, const std::string& n) { t.taskpool_name = n; })
      .def_property_readonly("taskpool_id", [](Taskpool& t) { return t.taskpool_id; })
      .def_property("priority", [](Taskpool& t) { return t.priority; }, [](Taskpool& t, int p) { taskpool_set_priority(&t, p); })
      .def_property("devices_mask", [](Taskpool& t) { return t.devices_index_mask; }, [](Taskpool& t, uint32_t m) { t.devices_index_mask = m; })
      .def_property("termdet", [](Taskpool& t) { return t.termdet_name; }, [](Taskpool& t, const std::string& n) { t.termdet_name = n; })
      .def_property_readonly("nb_tasks", [](Taskpool& t) { return t.nb_tasks.load(); })
      .def_property_readonly("nb_pending_actions", [](Taskpool& t) { return t.nb_pending_actions.load(); })
      // termination-detector counters (reference parsec_taskpool_update_nbtask /
      // runtime_actions); only meaningful on a monitored taskpool
      .def("addto_nb_tasks", [](Taskpool& t, int64_t d) { return t.tdm ? t.tdm->taskpool_addto_nb_tasks(&t, d) : (int64_t)0; })
      .def("addto_runtime_actions", [](Taskpool& t, int64_t d) { return t.tdm ? t.tdm->taskpool_addto_runtime_actions(&t, d) : (int64_t)0; })
      .def_property_readonly("completed", [](Taskpool& t) { return t.completed.load(); })
      .def_property_readonly("simulation_date", [](Taskpool& t) { return t.largest_simulation_date.load(); })
      .def("set_complete_callback", [](Taskpool& t, py::function f) {
        auto holder = std::make_shared<py::function>(f);
        t.on_complete = [holder](Taskpool*) {
          py::gil_scoped_acquire g;
          py::object r = (*holder)();
          return r.is_none() ? 0 : r.cast<int>();
        };
      })
      .def("set_enqueue_callback", [](Taskpool& t, py::function f) {
        auto holder = std::make_shared<py::function>(f);
        t.on_enqueue = [holder](Taskpool*) {
          py::gil_scoped_acquire g;
          py::object r = (*holder)();
          return r.is_none() ? 0 : r.cast<int>();
        };
      })
      .def("task_classes", [](Taskpool& t) {
        std::vector<std::string> out;
        for (auto* tc : t.task_classes) out.push_back(tc->name);
        return out;
      });
  m.def("taskpool_free", [](Taskpool* tp) { taskpool_free(tp); });
  m.def("compose", [](Taskpool* a, Taskpool* b) { return compose(a, b); }, py::return_value_policy::reference);
  m.def("taskpool_lookup", [](uint32_t id) { return taskpool_lookup(id); }, py::return_value_policy::reference);
  m.def("taskpool_sync_ids", []() { taskpool_sync_ids(); });

  py::class_<ptg::PtgTaskpool, Taskpool>(m, "PtgTaskpool")
      .def("set_global", &ptg::PtgTaskpool::set_global)
      .def("global_", &ptg::PtgTaskpool::global)
      .def("nb_task_classes", [](ptg::PtgTaskpool& t) { return t.classes.size(); })
      .def("count_tasks", [](ptg::PtgTaskpool& t, const std::string& name) {
        if (!t.finalized) t.finalize();
        int64_t n = 0;
        for (auto* tc : t.classes)
          if (tc->name == name) ptg::for_each_task(&t, tc, [&](const int32_t*) { ++n; });
        return n;
      });

  // ------------------------------------------------------------------ DTD
  py::class_<dtd::Tile>(m, "Tile")
      .def_property_readonly("rank", [](dtd::Tile& t) { return t.rank; })
      .def_property_readonly("key", [](dtd::Tile& t) { return t.key; })
      .def("data", [](dtd::Tile& t) -> py::object {
        if (!t.data) return py::none();
        DataCopy* c = data_pull_to_host(t.data);
        if (!c) return py::none();
        if (t.dc) if (auto* tm = dynamic_cast<TiledMatrix*>(t.dc)) return tile_view(c->device_private, tm->mtype, tm->mb, tm->nb, tm->elem_size);
        return py::array(py::dtype::of<uint8_t>(), {(py::ssize_t)t.data->nb_elts}, {1}, c->device_private, py::capsule(c->device_private, [](void*) {}));
      });

  py::class_<PyTask>(m, "Task")
      .def("arg", [](PyTask& p, int i) { return dtd_arg(p.t, i); })
      .def("value_int", [](PyTask& p, int i) { auto* a = static_cast<int32_t*>(dtd::task_arg(p.t, i)); return a ? (int64_t)*a : 0; })
      .def("value_int64", [](PyTask& p, int i) { auto* a = static_cast<int64_t*>(dtd::task_arg(p.t, i)); return a ? *a : 0; })
      .def("value_double", [](PyTask& p, int i) { auto* a = static_cast<double*>(dtd::task_arg(p.t, i)); return a ? *a : 0.0; })
      .def("ptr", [](PyTask& p, int i) { return (uintptr_t)dtd::task_arg(p.t, i); })
      .def_property_readonly("nb_args", [](PyTask& p) { return dtd::task_nb_args(p.t); })
      .def_property_readonly("seq", [](PyTask& p) { return static_cast<dtd::DtdTask*>(p.t)->seq; })
      .def_property_readonly("rank", [](PyTask& p) { return static_cast<dtd::DtdTask*>(p.t)->rank; })
      .def_property_readonly("name", [](PyTask& p) { return p.t->task_class->name; })
      .def_property_readonly("priority", [](PyTask& p) { return p.t->priority; })
      .def("user_trigger_termination", [](PyTask& p) { p.t->taskpool->tdm->user_trigger(p.t->taskpool); })
      .def("recursive_call", [](PyTask& p, Taskpool* inner) { return recursive_call(my_execution_stream(), p.t, inner); },
           "run `inner` as this task's body; return the result (HOOK_ASYNC) from the body");

  py::class_<dtd::DtdTaskClass>(m, "DtdTaskClass")
      .def_property_readonly("name", [](dtd::DtdTaskClass& c) { return c.name; })
      .def_property_readonly("nb_flows", [](dtd::DtdTaskClass& c) { return c.flows.size(); });

  py::class_<dtd::DtdTaskpool, Taskpool>(m, "DtdTaskpool")
      .def(py::init([]() { return new dtd::DtdTaskpool(); }))
      .def("task_class", [](dtd::DtdTaskpool& tp, const std::string& name, std::vector<std::pair<int, int>> params) { return tp.create_task_class(name, params); },
           py::return_value_policy::reference)
      .def("add_chore",
           [](dtd::DtdTaskpool& tp, dtd::DtdTaskClass* tc, int device, py::object fn, const std::string& builtin) {
             Hook cpu;
             std::function<int(GpuExecContext*, Task*)> gpu;
             if (!fn.is_none()) {
               auto holder = std::make_shared<py::object>(fn);
               cpu = [holder](ExecutionStream*, Task* t) {
                 py::gil_scoped_acquire g;
                 PyTask pt{t};
                 py::object r = (*holder)(pt);
                 return r.is_none() ? (int)HOOK_DONE : r.cast<int>();
               };
             }
             if (!builtin.empty()) gpu = builtin_dtd_gpu_body(builtin);
             return tp.add_chore(tc, (uint32_t)device, cpu, gpu);
           },
           py::arg("tc"), py::arg("device"), py::arg("fn") = py::none(), py::arg("builtin") = "")
      .def("insert_task",
           [](dtd::DtdTaskpool& tp, dtd::DtdTaskClass* tc, py::list args, int priority) {
             std::vector<dtd::Arg> a;
             std::vector<std::string> store;  // keep VALUE bytes alive during insertion
             store.reserve(args.size());
             for (auto item : args) {
               py::tuple tup = item.cast<py::tuple>();
               dtd::Arg x;
               x.op = tup[1].cast<int>();
               int op = x.op & dtd::OP_MASK;
               py::object o = tup[0];
               if (op == dtd::VALUE) {
                 if (py::isinstance<py::bytes>(o)) store.push_back(o.cast<std::string>());
                 else if (py::isinstance<py::float_>(o)) { double v = o.cast<double>(); store.emplace_back((const char*)&v, sizeof v); }
                 else { int64_t v = o.cast<int64_t>(); int32_t v32 = (int32_t)v; if (tup.size() > 2 && tup[2].cast<int>() == 8) store.emplace_back((const char*)&v, 8); else store.emplace_back((const char*)&v32, 4); }
                 x.ptr = store.back().data();
                 x.size = (int)store.back().size();
               } else if (op == dtd::SCRATCH) {
                 x.size = o.cast<int>();
               } else if (op == dtd::REF) {
                 x.ptr = (void*)o.cast<uintptr_t>();
               } else {
                 x.tile = o.is_none() ? nullptr : o.cast<dtd::Tile*>();
                 x.size = dtd::PASSED_BY_REF;
               }
               a.push_back(x);
             }
             py::gil_scoped_release rel;
             tp.insert_task(tc, priority, a);
           },
           py::arg("tc"), py::arg("args"), py::arg("priority") = 0)
      .def("tile_of", [](dtd::DtdTaskpool& tp, DataCollection* dc, uint64_t key) { return tp.tile_of(dc, key); }, py::return_value_policy::reference)
      .def("tile_new", [](dtd::DtdTaskpool& tp, size_t bytes, int rank) { return tp.tile_new(bytes, rank); }, py::return_value_policy::reference)
      .def("data_flush", [](dtd::DtdTaskpool& tp, dtd::Tile* t) { py::gil_scoped_release rel; return tp.data_flush(t); })
      .def("data_flush_all", [](dtd::DtdTaskpool& tp, DataCollection* dc) { py::gil_scoped_release rel; return tp.data_flush_all(dc); })
      .def("wait", [](dtd::DtdTaskpool& tp) { py::gil_scoped_release rel; return tp.wait(); })
      .def("close", [](dtd::DtdTaskpool& tp) { tp.release_hold(); }, "no more insertions: the taskpool may terminate once its tasks ran")
      .def_property("window", [](dtd::DtdTaskpool& tp) { return tp.window; }, [](dtd::DtdTaskpool& tp, int64_t w) { tp.window = w; })
      .def_property("threshold", [](dtd::DtdTaskpool& tp) { return tp.threshold; }, [](dtd::DtdTaskpool& tp, int64_t w) { tp.threshold = w; });

  // ----------------------------------------------------------- collections
  py::class_<DataCollection>(m, "DataCollection")
      .def_property_readonly("myrank", [](DataCollection& d) { return d.myrank; })
      .def_property_readonly("nodes", [](DataCollection& d) { return d.nodes; })
      .def_property_readonly("dc_id", [](DataCollection& d) { return d.dc_id; })
      .def("rank_of", [](DataCollection& d, std::vector<int64_t> idx) { return d.rank_of(idx.data(), (int)idx.size()); })
      .def("vpid_of", [](DataCollection& d, std::vector<int64_t> idx) { return d.vpid_of(idx.data(), (int)idx.size()); })
      .def("data_key", [](DataCollection& d, std::vector<int64_t> idx) { return d.data_key(idx.data(), (int)idx.size()); })
      .def("rank_of_key", &DataCollection::rank_of_key)
      .def("key_to_string", &DataCollection::key_to_string);

  py::class_<TiledMatrix, DataCollection>(m, "TiledMatrix")
      .def_readonly("mb", &TiledMatrix::mb)
      .def_readonly("nb", &TiledMatrix::nb)
      .def_readonly("lm", &TiledMatrix::lm)
      .def_readonly("ln", &TiledMatrix::ln)
      .def_readonly("mt", &TiledMatrix::mt)
      .def_readonly("nt", &TiledMatrix::nt)
      .def_readonly("lmt", &TiledMatrix::lmt)
      .def_readonly("lnt", &TiledMatrix::lnt)
      .def_readonly("mtype", &TiledMatrix::mtype)
      .def_readonly("nb_local_tiles", &TiledMatrix::nb_local_tiles)
      .def_readonly("storage_device", &TiledMatrix::storage_device)
      .def_property_readonly("storage_ptr", [](TiledMatrix& t) { return (uintptr_t)t.mat; })
      .def_property_readonly("storage_bytes", [](TiledMatrix& t) { return (size_t)t.nb_local_tiles * (size_t)t.bsiz * t.elem_size; })
      .def("local_index", &TiledMatrix::local_index)
      .def("data_write", [](TiledMatrix& t, const std::string& f) { py::gil_scoped_release rel; return t.data_write(f); })
      .def("data_read", [](TiledMatrix& t, const std::string& f) { py::gil_scoped_release rel; return t.data_read(f); })
      .def("tile_ptr", [](TiledMatrix& t, int64_t a, int64_t b) { return (uintptr_t)t.tile_ptr(a, b); })
      .def("tile", [](TiledMatrix& t, int64_t a, int64_t b) -> py::object {
        // column-major numpy view of the newest host copy of a local tile
        // (virtual data_of: views resolve to their origin's tiles)
        const int64_t idx[2] = {a, b};
        Data* d = t.data_of(idx, 2);
        if (!d) return py::none();
        DataCopy* c = data_pull_to_host(d);
        if (!c) return py::none();
        if (auto* st = dynamic_cast<SubTileMatrix*>(&t)) {  // strided view into the parent tile
          const size_t es = st->elem_size;
          return py::array(py::dtype(st->mtype == MATRIX_INTEGER ? "int32" : (st->mtype == MATRIX_FLOAT ? "float32" : "float64")),
                           {(py::ssize_t)st->tile_rows(a), (py::ssize_t)st->tile_cols(b)}, {(py::ssize_t)es, (py::ssize_t)(es * st->plda)},
                           c->device_private, py::capsule(c->device_private, [](void*) {}));
        }
        return tile_view(c->device_private, t.mtype, t.mb, t.nb, t.elem_size);
      })
      .def("mark_host_modified", [](TiledMatrix& t, int64_t a, int64_t b) {
        const int64_t idx[2] = {a, b};
        Data* d = t.data_of(idx, 2);
        if (!d) return;
        DataCopy* c = d->copy(0);
        if (!c) return;
        std::lock_guard<SpinLock> g(d->lock);
        c->version = d->newest_version() + 1;
        c->coherency_state = COHERENCY_OWNED;
        d->owner_device = 0;
      })
      .def("tile_rows", &TiledMatrix::tile_rows)
      .def("tile_cols", &TiledMatrix::tile_cols);

  py::class_<BlockCyclic, TiledMatrix>(m, "BlockCyclic")
      .def(py::init([](int mtype, int myrank, int64_t mb, int64_t nb, int64_t lm, int64_t ln, int P, int Q, int kp, int kq, int ip, int jq, int device, uintptr_t ptr, int nb_vp) {
             auto* bc = new BlockCyclic();
             bc->storage_device = device;
             bc->init(mtype, myrank, mb, nb, lm, ln, 0, 0, lm, ln, P, Q, kp, kq, ip, jq);
             bc->nb_vp = nb_vp;
             bc->allocate_storage((void*)ptr);
             return bc;
           }),
           py::arg("mtype"), py::arg("myrank"), py::arg("mb"), py::arg("nb"), py::arg("lm"), py::arg("ln"), py::arg("P") = 1, py::arg("Q") = 1,
           py::arg("kp") = 1, py::arg("kq") = 1, py::arg("ip") = 0, py::arg("jq") = 0, py::arg("device") = 0, py::arg("ptr") = 0, py::arg("nb_vp") = 1)
      .def_readonly("P", &BlockCyclic::P)
      .def_readonly("Q", &BlockCyclic::Q)
      .def_readonly("llm_tiles", &BlockCyclic::llm_tiles)
      .def_readonly("lln_tiles", &BlockCyclic::lln_tiles);

  // views (reference parsec_matrix_block_cyclic_kview, parsec_tiled_matrix_submatrix, subtile_desc_create)
  py::class_<KViewMatrix, TiledMatrix>(m, "KViewMatrix")
      .def(py::init([](BlockCyclic* o, int kp, int kq) { auto* v = new KViewMatrix(); v->init_view(o, kp, kq); return v; }), py::keep_alive<1, 2>(),
           py::arg("origin"), py::arg("kp"), py::arg("kq"))
      .def("origin_index", [](KViewMatrix& v, int64_t a, int64_t b) { return std::make_pair(v.map_m(a), v.map_n(b)); });
  py::class_<SubMatrixView, TiledMatrix>(m, "SubMatrixView")
      .def(py::init([](TiledMatrix* o, int64_t i, int64_t j, int64_t mm, int64_t nn) { auto* v = new SubMatrixView(); v->init_view(o, i, j, mm, nn); return v; }),
           py::keep_alive<1, 2>(), py::arg("origin"), py::arg("i"), py::arg("j"), py::arg("m"), py::arg("n"));
  py::class_<SubTileMatrix, TiledMatrix>(m, "SubTileMatrix")
      .def(py::init([](TiledMatrix* p, int64_t tm, int64_t tn, int64_t smb, int64_t snb) { auto* v = new SubTileMatrix(); v->init_subtile(p, tm, tn, smb, snb); return v; }),
           py::keep_alive<1, 2>(), py::arg("parent"), py::arg("tm"), py::arg("tn"), py::arg("smb"), py::arg("snb"))
      .def_readonly("plda", &SubTileMatrix::plda);

  py::class_<SymBlockCyclic, BlockCyclic>(m, "SymBlockCyclic")
      .def(py::init([](int mtype, int myrank, int64_t mb, int64_t nb, int64_t lm, int64_t ln, int P, int Q, int uplo, int device, uintptr_t ptr) {
             auto* bc = new SymBlockCyclic();
             bc->storage_device = device;
             bc->init_sym(mtype, myrank, mb, nb, lm, ln, 0, 0, lm, ln, P, Q, uplo);
             bc->allocate_storage((void*)ptr);
             return bc;
           }),
           py::arg("mtype"), py::arg("myrank"), py::arg("mb"), py::arg("nb"), py::arg("lm"), py::arg("ln"), py::arg("P") = 1, py::arg("Q") = 1,
           py::arg("uplo") = (int)MATRIX_LOWER, py::arg("device") = 0, py::arg("ptr") = 0);

  py::class_<TabularMatrix, TiledMatrix>(m, "TabularMatrix")
      .def(py::init([](int mtype, int myrank, int nodes, int64_t mb, int64_t nb, int64_t lm, int64_t ln, std::vector<int> ranks) {
             auto* t = new TabularMatrix();
             t->init_tab(mtype, myrank, nodes, mb, nb, lm, ln, ranks);
             t->allocate_storage(nullptr);
             return t;
           }),
           py::arg("mtype"), py::arg("myrank"), py::arg("nodes"), py::arg("mb"), py::arg("nb"), py::arg("lm"), py::arg("ln"), py::arg("ranks"));

  py::class_<VectorCyclic, TiledMatrix>(m, "VectorCyclic")
      .def(py::init([](int mtype, int myrank, int nodes, int64_t mb, int64_t lm, int dist, int P, int Q) {
             auto* v = new VectorCyclic();
             v->init_vec(mtype, myrank, nodes, mb, lm, dist, P, Q);
             v->allocate_storage(nullptr);
             return v;
           }),
           py::arg("mtype"), py::arg("myrank"), py::arg("nodes"), py::arg("mb"), py::arg("lm"), py::arg("dist") = 0, py::arg("P") = 1, py::arg("Q") = 1);

  py::class_<BandMatrix, TiledMatrix>(m, "BandMatrix")
      .def(py::init([](BlockCyclic* band, BlockCyclic* off, int bs) {
             auto* b = new BandMatrix();
             b->init_band(band, off, bs);
             return b;
           }),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>());

  py::class_<HashCollection, DataCollection>(m, "HashCollection")
      .def(py::init([](int myrank, int nodes) {
        auto* h = new HashCollection();
        h->myrank = (uint32_t)myrank;
        h->nodes = (uint32_t)nodes;
        dc_register_id(h);
        return h;
      }))
      .def("set_entry", [](HashCollection& h, uint64_t key, uint32_t rank, int32_t vp, uintptr_t ptr, size_t size) { h.set_entry(key, rank, vp, (void*)ptr, size); });

  // ---------------------------------------------------------------- algos
  m.def("dpotrf_new", [](TiledMatrix* A, int uplo) {
        auto* info = new int(0);
        auto* tp = algos::dpotrf_new(A, uplo, info);
        tp->destructor_hook = [info]() { delete info; };
        return py::make_tuple(py::cast(tp, py::return_value_policy::take_ownership), (uintptr_t)info);
      });
  m.def("trsm_inplace", [](int set) { return kern::trsm_inplace(set); }, py::arg("set") = -1,
        "Panel-solve W-GEMM in place (no B-tile copies; PARSEC_TRSM_INPLACE): 1 on, 0 off, < 0 query; returns the previous setting");
  m.def("dpotrf_fuse_syrk", [](int set) { return algos::dpotrf_fuse_syrk(set); }, py::arg("set") = -1,
        "SYRK(k-1,k) fused into POTRF(k) for new dpotrf_L.jdf taskpools (PARSEC_DPOTRF_FUSE_SYRK); returns the previous value");
  m.def("dpotrf_jdf_new", [](TiledMatrix* A) {
        auto* info = new int(0);
        auto* tp = algos::dpotrf_jdf_new(A, info);
        auto prev = tp->destructor_hook;
        tp->destructor_hook = [info, prev]() { if (prev) prev(); delete info; };
        return py::make_tuple(py::cast(tp, py::return_value_policy::take_ownership), (uintptr_t)info);
      }, "tiled Cholesky (lower) from the ptgpp-compiled algos/jdf/dpotrf_L.jdf; returns (taskpool, info address)");
  m.def("dgeqrf_jdf_new", [](TiledMatrix* A, TiledMatrix* T) { return algos::dgeqrf_jdf_new(A, T); }, py::arg("A"), py::arg("T"),
        py::return_value_policy::take_ownership, "Tiled QR from the ptgpp-compiled dgeqrf.jdf (GEQRT / TSQRT / UNMQR / TSMQR)");
  m.def("dgeqrf_new", [](TiledMatrix* A, TiledMatrix* T, int ib) { return algos::dgeqrf_new(A, T, ib); }, py::arg("A"), py::arg("T"), py::arg("ib") = 0,
        py::return_value_policy::take_ownership);
  m.def("dgeqrf_hqr_new", [](TiledMatrix* A, TiledMatrix* T, TiledMatrix* TT, int domain, int p_rows) { return algos::dgeqrf_hqr_new(A, T, TT, domain, p_rows); },
        py::arg("A"), py::arg("T"), py::arg("TT"), py::arg("domain") = 0, py::arg("p_rows") = 0, py::return_value_policy::take_ownership,
        "hierarchical tiled QR: TS domains of `domain` rows per process row (0: one flat TS chain per process row), TT binary trees over the domain heads and across process rows");
  py::class_<algos::StencilGrid, DataCollection>(m, "StencilGrid")
      .def(py::init([](int myrank, int nodes, int64_t nx, int64_t ny, int64_t nz, int bx, int by, int bz, int device) {
             auto* g = new algos::StencilGrid();
             g->init(myrank, nodes, nx, ny, nz, bx, by, bz, device);
             return g;
           }),
           py::arg("myrank"), py::arg("nodes"), py::arg("nx"), py::arg("ny"), py::arg("nz"), py::arg("bx"), py::arg("by"), py::arg("bz"), py::arg("device") = 0)
      .def_readonly("nblocks", &algos::StencilGrid::nblocks)
      .def("block_rank", &algos::StencilGrid::block_rank)
      .def("block_dims", [](algos::StencilGrid& g, int64_t b) { int x, y, z; g.block_dims(b, &x, &y, &z); return py::make_tuple(x, y, z); })
      .def("block", [](algos::StencilGrid& g, int64_t b, int parity) -> py::object {
        // host copy of block b's solution buffer (local blocks only), shape (ez, ey, ex)
        Data* d = g.data_of_key(g.key(0, parity, b, 0));
        if (!d) return py::none();
        DataCopy* c = data_pull_to_host(d);
        int x, y, z;
        g.block_dims(b, &x, &y, &z);
        std::vector<py::ssize_t> shape{z, y, x}, strides{(py::ssize_t)(8 * x * y), (py::ssize_t)(8 * x), 8};
        return py::array(py::dtype::of<double>(), shape, strides, c->device_private, py::capsule(c->device_private, [](void*) {}));
      });
  m.def("stencil3d_run", [](PxContext& c, algos::StencilGrid* g, int iters, double c0, double c1, bool gpu) {
        algos::Stencil3DResult r;
        {
          py::gil_scoped_release rel;
          r = algos::stencil3d_run(c.ctx, g, iters, c0, c1, gpu);
        }
        return py::make_tuple(r.seconds, r.points, r.final_parity);
      }, py::arg("ctx"), py::arg("grid"), py::arg("iters"), py::arg("c0") = 0.4, py::arg("c1") = 0.1, py::arg("gpu") = true);
  // ------------------------------------------------ collection operators
  m.def("apply_new", [](TiledMatrix* A, int uplo, py::function fn) {
        auto* keep = new py::function(fn);
        auto* tp = algos::apply_new(A, uplo, [keep](TiledMatrix* M, int64_t mm, int64_t nn, void* tile, void*) {
          py::gil_scoped_acquire g;
          (*keep)(mm, nn, tile_view(tile, M->mtype, M->mb, M->nb, M->elem_size));
        }, nullptr);
        tp->destructor_hook = [keep] { py::gil_scoped_acquire g; delete keep; };
        return (Taskpool*)tp;
      }, py::return_value_policy::take_ownership);
  m.def("map_new", [](TiledMatrix* src, TiledMatrix* dst, py::function fn) {
        auto* keep = new py::function(fn);
        auto* tp = algos::map_operator_new(src, dst, [keep, src, dst](const void* s, void* d, int64_t mm, int64_t nn, int64_t, int64_t) {
          py::gil_scoped_acquire g;
          (*keep)(tile_view(const_cast<void*>(s), src->mtype, src->mb, src->nb, src->elem_size), tile_view(d, dst->mtype, dst->mb, dst->nb, dst->elem_size), mm, nn);
        });
        tp->destructor_hook = [keep] { py::gil_scoped_acquire g; delete keep; };
        return (Taskpool*)tp;
      }, py::return_value_policy::take_ownership);
  auto reduce_binding = [](bool by_col) {
    return [by_col](TiledMatrix* A, TiledMatrix* res, py::object fn) {
      algos::ReduceOp op;
      py::function* keep = nullptr;
      if (py::isinstance<py::str>(fn) && fn.cast<std::string>() == "sum") {
        const int64_t ld = A->mb;
        op = [ld](const void* in, void* io, int64_t rows, int64_t cols, bool first) {
          const double* a = static_cast<const double*>(in);
          double* r = static_cast<double*>(io);
          for (int64_t c = 0; c < cols; ++c)
            for (int64_t i = 0; i < rows; ++i) r[i + c * ld] = (first ? 0.0 : r[i + c * ld]) + a[i + c * ld];
        };
      } else {
        keep = new py::function(fn.cast<py::function>());
        op = [keep, A](const void* in, void* io, int64_t, int64_t, bool first) {
          py::gil_scoped_acquire g;
          (*keep)(tile_view(const_cast<void*>(in), A->mtype, A->mb, A->nb, A->elem_size), tile_view(io, A->mtype, A->mb, A->nb, A->elem_size), first);
        };
      }
      auto* tp = by_col ? algos::reduce_col_new(A, res, op) : algos::reduce_row_new(A, res, op);
      if (keep) tp->destructor_hook = [keep] { py::gil_scoped_acquire g; delete keep; };
      return (Taskpool*)tp;
    };
  };
  m.def("reduce_col_new", reduce_binding(true), py::return_value_policy::take_ownership);
  m.def("reduce_row_new", reduce_binding(false), py::return_value_policy::take_ownership);
  m.def("broadcast_new", [](TiledMatrix* A, int64_t rm, int64_t rn, TiledMatrix* dst) { return (Taskpool*)algos::broadcast_new(A, rm, rn, dst); },
        py::return_value_policy::take_ownership);
  m.def("redistribute", [](PxContext& c, TiledMatrix* src, TiledMatrix* dst, int64_t size_row, int64_t size_col, int64_t disi_src, int64_t disj_src, int64_t disi_dst,
                           int64_t disj_dst, const std::string& method) {
        py::gil_scoped_release rel;
        if (method == "dtd") return algos::redistribute(c.ctx, src, dst, size_row, size_col, disi_src, disj_src, disi_dst, disj_dst);
        if (method != "ptg") throw std::invalid_argument("redistribute: method is 'ptg' or 'dtd'");
        return algos::redistribute_ptg(c.ctx, src, dst, size_row, size_col, disi_src, disj_src, disi_dst, disj_dst);
      }, py::arg("ctx"), py::arg("src"), py::arg("dst"), py::arg("size_row"), py::arg("size_col"), py::arg("disi_src"), py::arg("disj_src"),
      py::arg("disi_dst"), py::arg("disj_dst"), py::arg("method") = "ptg",
      "copy a window between two tiled matrices (PTG redistribute.jdf / redistribute_reshuffle.jdf, or the DTD form)");
  m.def("redistribute_new", [](TiledMatrix* src, TiledMatrix* dst, int64_t size_row, int64_t size_col, int64_t disi_src, int64_t disj_src, int64_t disi_dst,
                               int64_t disj_dst) {
        auto* tp = algos::redistribute_new(src, dst, size_row, size_col, disi_src, disj_src, disi_dst, disj_dst);
        if (!tp) throw std::invalid_argument("redistribute_new: invalid window");
        return (Taskpool*)tp;
      }, py::return_value_policy::take_ownership);
  m.def("diag_band_to_rect_new", [](TiledMatrix* A, TiledMatrix* B, int mt, int nt, int mb, int nb) {
        auto* tp = algos::diag_band_to_rect_new(A, B, mt, nt, mb, nb, A->elem_size);
        if (!tp) throw std::invalid_argument("diag_band_to_rect_new: incompatible shapes");
        return (Taskpool*)tp;
      }, py::return_value_policy::take_ownership);
  m.def("dgemm_new", [](double alpha, TiledMatrix* A, TiledMatrix* B, double beta, TiledMatrix* C, int transB) { return (Taskpool*)algos::dgemm_new(alpha, A, B, beta, C, transB); },
        py::arg("alpha"), py::arg("A"), py::arg("B"), py::arg("beta"), py::arg("C"), py::arg("transB") = 0, py::return_value_policy::take_ownership);
  m.def("dtd_dgemm", [](PxContext& c, double alpha, TiledMatrix* A, TiledMatrix* B, double beta, TiledMatrix* C, bool gpu) {
        py::gil_scoped_release rel;
        return algos::dtd_dgemm(c.ctx, alpha, A, B, beta, C, gpu);
      }, py::arg("ctx"), py::arg("alpha"), py::arg("A"), py::arg("B"), py::arg("beta"), py::arg("C"), py::arg("gpu") = false);
  m.def("read_int", [](uintptr_t p) { return *reinterpret_cast<int*>(p); });

  // --------------------------------------------------------------- devices
  m.attr("DATA_ADVICE_PREFETCH") = (int)DATA_ADVICE_PREFETCH;
  m.attr("DATA_ADVICE_PREFERRED_DEVICE") = (int)DATA_ADVICE_PREFERRED_DEVICE;
  m.attr("DATA_ADVICE_WARMUP") = (int)DATA_ADVICE_WARMUP;
  m.def("data_advise", [](TiledMatrix* A, int64_t m, int64_t n, int device, int advice) {
        const int64_t idx[2] = {m, n};
        return data_advise_on_device(A->data_of(idx, 2), device, advice);
      }, "advise the runtime about tile (m, n): DATA_ADVICE_PREFETCH copies it to the device ahead of use, "
         "DATA_ADVICE_PREFERRED_DEVICE steers tasks writing it to that device (reference parsec_advise_data_on_device)");
  m.def("devices", []() {
    py::list out;
    for (auto* d : DeviceRegistry::instance().devices) {
      if (!d) continue;
      py::dict e;
      e["index"] = d->device_index;
      e["name"] = d->name;
      e["type"] = d->type;
      e["gflops_fp64"] = d->gflops_fp64;
      e["weight"] = d->gflops_weight;
      e["executed_tasks"] = d->stats.executed_tasks.load();
      e["ms_complete"] = d->stats.ns_complete.load() / 1e6;
      e["ms_complete_max"] = d->stats.ns_complete_max.load() / 1e6;
      e["ms_launch"] = d->stats.ns_launch.load() / 1e6;
      e["kernel_launches"] = d->stats.kernel_launches.load();
      e["early_released"] = d->stats.early_released.load();
      e["batched_tasks"] = d->stats.batched_tasks.load();
      e["bytes_in"] = d->stats.bytes_in.load();
      e["bytes_out"] = d->stats.bytes_out.load();
      e["bytes_d2d"] = d->stats.bytes_d2d.load();
      e["data_faults"] = d->stats.data_faults.load();
      e["w2r_tasks"] = d->stats.w2r_tasks.load();
      e["prefetches"] = d->stats.prefetches.load();
      e["staged_tasks"] = d->stats.staged_tasks.load();
      e["ms_stage_wait"] = d->stats.ns_stage_wait.load() / 1e6;
      e["copies_timed"] = d->stats.copies_timed.load();
      e["ms_copy_busy"] = d->stats.ns_copy_busy.load() / 1e6;
      e["ms_copy_window"] = (d->stats.ns_copy_last.load() - d->stats.ns_copy_first.load()) / 1e6;
      out.append(e);
    }
    return out;
  });
  m.def("nb_gpus", []() { return DeviceRegistry::instance().nb_gpus(); });
  m.def("first_gpu_device_index", &first_gpu_device_index);
  m.def("device_alloc", [](int dev, size_t bytes) { return (uintptr_t)device_alloc(dev, bytes); });
  m.def("device_free", [](int dev, uintptr_t p) { device_free(dev, (void*)p); });
  m.def("device_memcpy", [](int dd, uintptr_t dst, int sd, uintptr_t src, size_t n) { return device_memcpy(dd, (void*)dst, sd, (const void*)src, n); });
  m.def("trsm_inverse_mode", [](int mode, double limit) { return trsm_inverse_mode(mode, limit); }, py::arg("mode") = -1, py::arg("limit") = 0.0,
        "Tile-Cholesky panel solve: 0 through W = L^-1, 1 auto (substitution when max|L| max|W| > limit), 2 substitution; returns the previous mode");
  m.def("trsm_inverse_limit", []() { return trsm_inverse_limit(); });
  m.def("trsm_estimate_route", [](int on) { return kern::trsm_estimate_route(on); }, py::arg("on") = -1,
        "Auto panel solve: 1 decide on the host from the estimate the local POTRF published, 0 device-side gate only; returns the previous setting");
  m.def("trsm_estimate_lookup", [](uintptr_t p) { return kern::trsm_estimate_lookup((const void*)p); },
        "Published panel estimate keyed by the W address p on the current device (0 = unknown)");
  m.def("trsm_estimate_known", []() { return kern::trsm_estimate_known(); }, "W addresses with a published panel estimate (current device)");
  m.def("device_cache_alloc", [](int dev, size_t bytes) { return (uintptr_t)device_cache_alloc(dev, bytes); }, "Carve a buffer from a GPU's tile-cache zone");
  m.def("device_cache_free", [](int dev, uintptr_t p) { return device_cache_free(dev, (void*)p); });
  m.def("trsm_estimate_stats", [](bool reset) {
    uint64_t v[3];
    kern::trsm_estimate_stats(v, reset);
    return py::make_tuple(v[0], v[1], v[2]);
  }, py::arg("reset") = false, "(published by POTRF, decided on the host, left to the device gate)");
  m.def("device_memcpy_stats", [](bool reset) {
    uint64_t b[3];
    device_memcpy_stats(b, reset);
    py::dict d;
    d["h2d"] = b[0];
    d["d2h"] = b[1];
    d["d2d"] = b[2];
    return d;
  }, py::arg("reset") = false, "Bytes moved by the blocking device_memcpy helper (H2D / D2H / D2D), optionally reset");

  // raw kernels (tests): descriptors built in python, device pointers as ints
  m.def("kernel_dgemm", [](uintptr_t A, uintptr_t B, uintptr_t C, int mm, int nn, int kk, int lda, int ldb, int ldc, double alpha, double beta, int transB, int lower, uintptr_t stream) {
    GemmDesc g{(const double*)A, (const double*)B, (double*)C, mm, nn, kk, lda, ldb, ldc, alpha, beta, 0, (uint8_t)transB, (uint8_t)lower, 0};
    return parsec_amd_dgemm_batch(&g, 1, (void*)stream);
  });
  m.def("kernel_dgemm_batch", [](std::vector<std::tuple<uintptr_t, uintptr_t, uintptr_t, int, int, int, int, int, int, double, double, int, int>> ds, uintptr_t stream) {
    std::vector<GemmDesc> v;
    for (auto& d : ds) {
      GemmDesc g{(const double*)std::get<0>(d), (const double*)std::get<1>(d), (double*)std::get<2>(d), std::get<3>(d), std::get<4>(d), std::get<5>(d), std::get<6>(d), std::get<7>(d), std::get<8>(d), std::get<9>(d), std::get<10>(d), 0, (uint8_t)std::get<11>(d), (uint8_t)std::get<12>(d), 0};
      v.push_back(g);
    }
    return parsec_amd_dgemm_batch(v.data(), (int)v.size(), (void*)stream);
  });
  m.def("kernel_gemm_tile_policy", [](int p) { return parsec_amd_gemm_tile_policy(p); });
  m.def("kernel_gemm_splitk", [](int on) { return parsec_amd_gemm_splitk(on); }, "split-K tail of the 128x128 grouped DGEMM: 1 on, 0 off, -1 query; returns the previous setting");
  m.def("cpu_capability", []() {
    const CpuCapability c = cpu_capability();
    py::dict d;
    d["model"] = c.model;
    d["isa"] = c.isa();
    d["ghz"] = c.ghz;
    d["dp_flops_per_cycle"] = c.dp_flops_per_cycle;
    return d;
  }, "CPU model, widest vector ISA, clock and peak fp64 flops per cycle and core (/proc/cpuinfo, cpufreq)");
  m.def("kernel_potrf_stamps", []() {
    std::vector<long long> v(16, 0);
    if (parsec_amd_potrf_stamps(v.data()) != 0) v.clear();
    return v;
  });
  m.def("kernel_potrf_steps", [](int on) { return parsec_amd_potrf_steps(on); }, "tile POTRF: 1 = n/64 + 1 fused step launches, 0 = 3 launches per 64 columns, -1 query; returns the previous setting");
  m.def("kernel_dtrsm", [](uintptr_t L, uintptr_t B, int mm, int nn, int ldl, int ldb, uintptr_t stream) {
    TrsmDesc t;
    t.L = (const double*)L; t.B = (double*)B; t.m = mm; t.n = nn; t.ldl = ldl; t.ldb = ldb; t.trans = 1;
    return parsec_amd_dtrsm_batch(&t, 1, (void*)stream);
  });
  m.def("kernel_qr_panel", [](uintptr_t A1, int lda1, uintptr_t A2, int lda2, uintptr_t T, int ldt, uintptr_t V, int m1, int m2, int n, uintptr_t stream) {
    QrPanelDesc q{};
    q.A1 = (double*)A1; q.lda1 = lda1; q.A2 = (double*)A2; q.lda2 = lda2; q.T = (double*)T; q.ldt = ldt; q.Vcopy = (double*)V;
    q.m1 = m1; q.m2 = m2; q.n = n;
    return parsec_amd_qr_panel(&q, 1, (void*)stream);
  });
  m.def("kernel_qr_profile", []() {
    std::vector<unsigned long long> v(32, 0);
    if (parsec_amd_qr_profile(v.data()) != 0) v.clear();
    return v;
  });
  m.def("kernel_qr_apply", [](uintptr_t V, int ldv, uintptr_t T, int ldt, uintptr_t A1, int lda1, uintptr_t A2, int lda2, int m2, int n, int ncols, uintptr_t ws, uintptr_t stream) {
    QrApplyDesc q{};
    q.V = (const double*)V; q.ldv = ldv; q.T = (const double*)T; q.ldt = ldt; q.A1 = (double*)A1; q.lda1 = lda1; q.A2 = (double*)A2; q.lda2 = lda2;
    q.m2 = m2; q.n = n; q.ncols = ncols;
    return parsec_amd_qr_apply(&q, 1, (void*)ws, (void*)stream);
  });
  // batched block-reflector applications (one grouped launch per GEMM phase):
  // tuples (V, ldv, T, ldt, A1, lda1, A2, lda2, m2, n, ncols); ws sized by kernel_qr_apply_ws
  m.def("kernel_qr_apply_batch", [](const std::vector<std::tuple<uintptr_t, int, uintptr_t, int, uintptr_t, int, uintptr_t, int, int, int, int>>& ds, uintptr_t ws, uintptr_t stream) {
    std::vector<QrApplyDesc> v;
    for (const auto& d : ds) {
      QrApplyDesc q{};
      q.V = (const double*)std::get<0>(d); q.ldv = std::get<1>(d); q.T = (const double*)std::get<2>(d); q.ldt = std::get<3>(d);
      q.A1 = (double*)std::get<4>(d); q.lda1 = std::get<5>(d); q.A2 = (double*)std::get<6>(d); q.lda2 = std::get<7>(d);
      q.m2 = std::get<8>(d); q.n = std::get<9>(d); q.ncols = std::get<10>(d);
      v.push_back(q);
    }
    return parsec_amd_qr_apply(v.data(), (int)v.size(), (void*)ws, (void*)stream);
  });
  m.def("kernel_qr_apply_ws", [](int count, int n, int ncols) {
    std::vector<QrApplyDesc> v(count);
    for (auto& q : v) { q.n = n; q.ncols = ncols; }
    return parsec_amd_qr_apply_ws(v.data(), count);
  });
  m.def("kernel_dpotrf", [](uintptr_t A, int n, int lda, uintptr_t info, uintptr_t stream) { return parsec_amd_dpotrf_tile((double*)A, n, lda, (int*)info, (void*)stream); });
  m.def("kernel_dpotrf_w", [](uintptr_t A, int n, int lda, uintptr_t info, uintptr_t W, int ldw, uintptr_t stream, bool pack) {
    return parsec_amd_dpotrf_tile_w((double*)A, n, lda, (int*)info, (double*)W, ldw, (void*)stream, pack ? 1 : 0);
  }, py::arg("A"), py::arg("n"), py::arg("lda"), py::arg("info"), py::arg("W"), py::arg("ldw"), py::arg("stream"), py::arg("pack") = false,
     "Tile POTRF writing W = L^-1 (pack: W's strict upper triangle holds L^T, the packed panel tile)");
  // descriptors (B, W, m, n, ldb, ldw[, packed]): packed W = the packed panel
  // tile, which also provides L for the substitution routes
  m.def("kernel_trsm_w_batch", [](std::vector<py::tuple> ds, uintptr_t stream) {
    std::vector<TrsmGemmDesc> v;
    for (auto& d : ds) {
      TrsmGemmDesc t{(double*)d[0].cast<uintptr_t>(), (const double*)d[1].cast<uintptr_t>(), d[2].cast<int>(), d[3].cast<int>(), d[4].cast<int>(), d[5].cast<int>()};
      if (d.size() > 6 && d[6].cast<bool>()) {
        t.packed = 1;
        t.L = t.W;
        t.ldl = t.ldw;
      }
      v.push_back(t);
    }
    return parsec_amd_trsm_w_batch(v.data(), (int)v.size(), (void*)stream);
  });

  // ------------------------------------------------------------- profiling
  m.def("profiling_dump", [](const std::string& f) { return profiling_dump(f); });
  m.def("profiling_enabled", &profiling_enabled);
  m.def("pins_counters", []() { return pins_counters(); });
  m.def("properties", []() { return properties_snapshot(); });
  m.def("properties_set", &properties_set);
  m.def("properties_dump_shm", &properties_dump_shm);
  m.def("history", []() { return history_dump(); });

  // ------------------------------------------------------------------ comm
  m.def("comm_init", [](int rank, int size, const std::string& job, int gpu) { py::gil_scoped_release rel; return comm_init(rank, size, job, gpu); });
  m.def("comm_fini", []() { py::gil_scoped_release rel; comm_fini(); });
  m.def("topology", []() {
    py::dict d;
    py::list cpus;
    for (auto& c : topology_cpus()) {
      py::dict e;
      e["cpu"] = c[0]; e["package"] = c[1]; e["numa"] = c[2]; e["l2"] = c[3]; e["l3"] = c[4];
      cpus.append(e);
    }
    d["cpus"] = cpus;
    d["numa_distances"] = topology_numa_distances();
    return d;
  }, "hwloc-style view of the allowed CPUs (package, NUMA node, shared L2 / L3) and NUMA distances");
  m.def("comm_stats", []() { py::dict d; for (auto& kv : comm_stats()) d[py::str(kv.first)] = kv.second; return d; });
  m.def("comm_barrier", []() { py::gil_scoped_release rel; return comm_barrier(); });
  m.def("comm_rank", &comm_rank);
  m.def("comm_size", &comm_size);
  m.def("comm_device_plane", []() { return std::string(comm_device_plane_name()); });
  m.def("comm_bytes_by_peer", &comm_bytes_by_peer, "IPC payload bytes this rank pulled from each peer (xGMI link by link)");
  m.def("comm_pull_routes", &comm_pull_routes, "Pull route per peer: 0 copy engine, 1 copy kernel, 3 multi-source gather kernel");
  m.def("comm_probe_table", &comm_probe_table, "This rank's IPC start-up probe per peer: (bits: 1 open, 2 copy-engine pull, 4 copy kernel, 8 host read; 0 = ok, open attempts)");
  m.def("comm_plane_status", &comm_plane_status, "0, or the first failing step of this rank's IPC plane start-up (-1x set-up, -2x open of peer x, -4x copy from peer x, -6x bytes from peer x, -7 another rank failed)");
  m.def("comm_allreduce_max", [](uint32_t v) { py::gil_scoped_release rel; return comm_allreduce_max_u32(v); });
}
