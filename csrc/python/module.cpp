// pybind11 bindings: the native miint runtime + kernels as `cuda_v_mpi_amd._miint`.
//
// Device memory crosses the boundary as integer addresses (torch.Tensor.data_ptr()) and
// streams as integer handles (torch.cuda.Stream.cuda_stream), so the module has no libtorch
// ABI dependency and no hipify step; it links only libamdhip64 and librccl.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <cstdint>
#include <string>

#include "miint/comm.hpp"
#include "miint/expr.hpp"
#include "miint/fast_trig.hpp"
#include "miint/host.hpp"
#include "miint/integrator.hpp"
#include "miint/kernels.hpp"
#include "miint/oracle.hpp"
#include "miint/runtime.hpp"
#include "miint/selftest.hpp"
#include "miint/table2d.hpp"
#include "miint/trace.hpp"
#include "miint/trainscan.hpp"

namespace py = pybind11;
using namespace miint;

namespace {

template <typename T>
T* ptr(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

RiemannParams make_params(int integrand, double a, double h, double off, uint64_t i_begin,
                          uint64_t n, const std::vector<double>& coef, double p0, double p1) {
  RiemannParams p{};
  p.a = a;
  p.h = h;
  p.off = off;
  p.i_begin = i_begin;
  p.n = n;
  p.integrand = integrand;
  MIINT_CHECK(coef.size() <= static_cast<size_t>(kMaxPolyCoeffs), "too many coefficients");
  p.ncoef = static_cast<int>(coef.size());
  for (size_t i = 0; i < coef.size(); ++i) p.coef[i] = coef[i];
  p.p0 = p0;
  p.p1 = p1;
  return p;
}

}  // namespace

static const char* scan_algo_name(ScanAlgo a) {
  return a == ScanAlgo::kFused ? "fused" : a == ScanAlgo::kOnePass ? "onepass" : "lookback";
}
static ScanAlgo scan_algo_of(const std::string& s) {
  MIINT_CHECK(s == "fused" || s == "lookback" || s == "onepass",
              "algo must be onepass|fused|lookback");
  return s == "fused" ? ScanAlgo::kFused : s == "onepass" ? ScanAlgo::kOnePass : ScanAlgo::kLookback;
}

PYBIND11_MODULE(_miint, m) {
  m.doc() = "miint: MI355X-native numerical integration (HIP/gfx950 kernels, RCCL, hipGraph)";
  py::register_exception<miint::Error>(m, "MiintError", PyExc_RuntimeError);
  install_crash_handler_from_env();

  // ------------------------------------------------------------------ enums
  py::enum_<Integrand>(m, "Integrand")
      .value("pi4", Integrand::kPi4)
      .value("sin", Integrand::kSin)
      .value("poly", Integrand::kPoly)
      .value("train", Integrand::kTrainVel)
      .value("table", Integrand::kTable);
  py::enum_<Rule>(m, "Rule").value("left", Rule::kLeft).value("mid", Rule::kMid).value("right", Rule::kRight);
  py::enum_<DType>(m, "DType")
      .value("fp64", DType::kF64)
      .value("fp32", DType::kF32)
      .value("fp32acc", DType::kF32Acc32);
  py::enum_<DivMode>(m, "DivMode")
      .value("series", DivMode::kSeries)
      .value("ieee", DivMode::kIeee)
      .value("series_direct", DivMode::kSeriesDirect)
      .value("series_exact", DivMode::kSeriesExact);

  m.attr("TICKET_WORDS") = kTicketWords;
  m.attr("UNSET_SLOT_WORD") = kUnsetSlotWord;
  m.def("fill_unset_slots", [](uintptr_t p, size_t count, uintptr_t s) {
    fill_unset_slots(ptr<double>(p), count, stream(s));
  });
  m.attr("RIEMANN_TILE") = kRiemannTile;
  m.attr("RIEMANN_BLOCK") = kRiemannBlock;
  m.def("series_ok", &series_ok);
  m.def("series_ok_f32", &series_ok_f32);
  m.def("integrand_scale", &integrand_scale);

  // ------------------------------------------------------------------ devices
  m.def("device_count", &device_count);
  m.def("device_info", [](int d) {
    DeviceInfo i = device_info(d);
    py::dict r;
    r["index"] = i.index;
    r["name"] = i.name;
    r["arch"] = i.arch;
    r["num_cus"] = i.num_cus;
    r["clock_khz"] = i.clock_khz;
    r["total_mem"] = i.total_mem;
    r["l2_bytes"] = i.l2_bytes;
    return r;
  });
  m.def("set_device", &set_device);
  m.def("device_synchronize", []() { MIINT_HIP(hipDeviceSynchronize()); });
  // Host wait policy of the current device (hipDeviceSchedule*): "spin" polls the completion
  // signal (lowest wake-up latency, one busy core per waiting thread), "yield", "blocking"
  // (interrupt), "auto" (the runtime's default).
  m.def("set_device_flags", [](const std::string& mode) {
    unsigned f = hipDeviceScheduleAuto;
    if (mode == "spin") f = hipDeviceScheduleSpin;
    else if (mode == "yield") f = hipDeviceScheduleYield;
    else if (mode == "blocking") f = hipDeviceScheduleBlockingSync;
    else if (mode != "auto") throw std::invalid_argument("spin|yield|blocking|auto");
    MIINT_HIP(hipSetDeviceFlags(f));
  });
  m.def("get_device_flags", []() {
    unsigned f = 0;
    MIINT_HIP(hipGetDeviceFlags(&f));
    return f;
  });
  m.def("process_start_seconds", &process_start_seconds);
  m.def("enable_tracing", &enable_tracing, py::arg("on"),
        "roctx ranges around runtime phases (MIINT_ROCTX=1)");
  m.def("tracing_enabled", &tracing_enabled);
  m.def("trace_mark", &trace_mark);
  m.def("wait_with_timeout", [](uintptr_t s, double timeout_s) {
    py::gil_scoped_release nogil;
    return wait_with_timeout(stream(s), timeout_s, nullptr);
  });
  m.def("wall_seconds", &wall_seconds);

  // ------------------------------------------------------------------ comm
  py::class_<Comm>(m, "Communicator")
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("world", &Comm::world)
      .def_property_readonly("device", &Comm::device)
      .def_property_readonly("kind", [](const Comm& c) { return std::string(c.kind()); })
      .def_property_readonly("transport_world", &Comm::transport_world,
                             "ranks the transport reports (ncclCommCount for RCCL)")
      .def("allreduce_sum", [](const Comm& c, uintptr_t send, uintptr_t recv, size_t count,
                               uintptr_t s) {
             py::gil_scoped_release nogil;  // loopback collectives barrier across threads
             c.allreduce_sum(ptr<double>(send), ptr<double>(recv), count, stream(s));
           })
      .def("allgather", [](const Comm& c, uintptr_t send, uintptr_t recv, size_t count,
                           uintptr_t s) {
             py::gil_scoped_release nogil;
             c.allgather(ptr<double>(send), ptr<double>(recv), count, stream(s));
           })
      .def("broadcast", [](const Comm& c, uintptr_t buf, size_t count, int root, uintptr_t s) {
        py::gil_scoped_release nogil;
        c.broadcast(ptr<double>(buf), count, root, stream(s));
      })
      .def("reduce_sum", [](const Comm& c, uintptr_t send, uintptr_t recv, size_t count,
                            int root, uintptr_t s) {
        py::gil_scoped_release nogil;
        c.reduce_sum(ptr<double>(send), ptr<double>(recv), count, root, stream(s));
      })
      .def("check_async", &Comm::check_async);
  py::class_<RcclComm, Comm>(m, "Comm")
      .def(py::init([](py::bytes id, int rank, int world, int device) {
             return new RcclComm(std::string(id), rank, world, device);
           }),
           py::arg("unique_id"), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def_static("version", &RcclComm::version);
  py::class_<LoopbackComm, Comm>(m, "LoopbackComm");
  py::class_<LoopbackGroup, std::shared_ptr<LoopbackGroup>>(m, "LoopbackGroup",
      "W logical ranks on one device (test transport; drive rank r from its own thread)")
      .def(py::init(&LoopbackGroup::create), py::arg("world"), py::arg("device") = 0,
           py::arg("timeout_s") = 120.0)
      .def_property_readonly("world", &LoopbackGroup::world)
      .def_property_readonly("device", &LoopbackGroup::device)
      .def("comm", &LoopbackGroup::comm, py::arg("rank"), py::return_value_policy::reference_internal)
      .def("barrier", &LoopbackGroup::barrier, py::arg("rank"), py::call_guard<py::gil_scoped_release>())
      .def("mark_broken", &LoopbackGroup::mark_broken)
      .def_property_readonly("broken", &LoopbackGroup::broken)
      .def_property_readonly("collectives", &LoopbackGroup::collectives)
      .def_property_readonly("graph_launches", &LoopbackGroup::graph_launches);
  m.def(
      "rendezvous_unique_id",
      [](const std::string& addr, int port, int rank, int world, double timeout_s) {
        std::string id;
        {
          py::gil_scoped_release rel;  // rank 0 blocks in accept() until the others connect
          id = rendezvous_unique_id(addr, port, rank, world, timeout_s);
        }
        return py::bytes(id);  // 128 raw bytes, not text
      },
      py::arg("addr"), py::arg("port"), py::arg("rank"), py::arg("world"),
      py::arg("timeout_s") = 120.0);
  // RCCL transport evidence (miint/comm.hpp): which transport the ranks' connections use
  auto transport_dict = [](const RcclTransport& t) {
    py::dict d;
    d["transport"] = t.transport;
    d["nranks"] = t.nranks;
    d["nnodes"] = t.nnodes;
    d["local_ranks"] = t.local_ranks;
    d["connections"] = t.connections;
    d["comms"] = t.comms;
    d["uses_net"] = t.uses_net();
    d["log"] = t.log;
    return d;
  };
  m.def("parse_rccl_log", [transport_dict](const std::string& text) {
    return transport_dict(parse_rccl_log(text));
  });
  m.def("capture_rccl_log", &capture_rccl_log,
        "route RCCL's INIT log into a per-process file (call before the first RCCL call)");
  m.def("rccl_log_path", &rccl_log_path);
  m.def("rccl_transport", [transport_dict]() { return transport_dict(rccl_transport()); });
  m.def(
      "transport_error",
      [](const std::string& log_text, int world, int local_world, bool share) {
        return transport_error(parse_rccl_log(log_text), world, local_world, share);
      },
      "the native CLIs' fail-closed transport verdict on an RCCL INIT log (\"\" = ok)",
      py::arg("log_text"), py::arg("world"), py::arg("local_world"), py::arg("share"));

  // ------------------------------------------------------------------ Riemann plan
  py::class_<RiemannConfig>(m, "RiemannConfig")
      .def(py::init<>())
      .def_readwrite("integrand", &RiemannConfig::integrand)
      .def_readwrite("a", &RiemannConfig::a)
      .def_readwrite("b", &RiemannConfig::b)
      .def_readwrite("n", &RiemannConfig::n)
      .def_readwrite("rule", &RiemannConfig::rule)
      .def_readwrite("dtype", &RiemannConfig::dtype)
      .def_readwrite("div", &RiemannConfig::div)
      .def_readwrite("coef", &RiemannConfig::coef)
      .def_readwrite("p0", &RiemannConfig::p0)
      .def_readwrite("p1", &RiemannConfig::p1)
      .def_readwrite("table", &RiemannConfig::table)
      .def_readwrite("grid", &RiemannConfig::grid)
      .def_readwrite("block", &RiemannConfig::block)
      .def_readwrite("waves_per_cu", &RiemannConfig::waves_per_cu)
      .def_readwrite("fused", &RiemannConfig::fused)
      .def_readwrite("slots", &RiemannConfig::slots)
      .def_readwrite("bucket", &RiemannConfig::bucket)
      .def_readwrite("rank", &RiemannConfig::rank)
      .def_readwrite("world", &RiemannConfig::world)
      .def_readwrite("force_collective", &RiemannConfig::force_collective)
      .def_readwrite("step_streams", &RiemannConfig::step_streams)
      .def_readwrite("multistep", &RiemannConfig::multistep)
      .def_readwrite("slice_rank", &RiemannConfig::slice_rank)
      .def_readwrite("slice_world", &RiemannConfig::slice_world)
      .def_readwrite("timeout_s", &RiemannConfig::timeout_s)
      .def_readwrite("host_direct", &RiemannConfig::host_direct)
      .def_readwrite("close", &RiemannConfig::close)
      .def_readwrite("allreduce_to_host", &RiemannConfig::allreduce_to_host)
      .def_readwrite("chain", &RiemannConfig::chain);

  py::class_<RiemannPlan>(m, "RiemannPlan")
      .def(py::init<const RiemannConfig&, int, const Comm*>(), py::arg("config"),
           py::arg("device"), py::arg("comm") = nullptr, py::keep_alive<1, 4>())
      .def_property_readonly("device", &RiemannPlan::device)
      .def_property_readonly("rank", &RiemannPlan::rank)
      .def_property_readonly("world", &RiemannPlan::world)
      .def("step_streams", &RiemannPlan::step_streams, py::arg("nsteps"))
      .def_property_readonly("begin", &RiemannPlan::begin)
      .def_property_readonly("count", &RiemannPlan::count)
      .def_property_readonly("h", &RiemannPlan::h)
      .def_property_readonly("scale", &RiemannPlan::scale)
      .def_property_readonly("grid", [](const RiemannPlan& p) { return p.shape().grid; })
      .def_property_readonly("block", [](const RiemannPlan& p) { return p.shape().block; })
      .def_property_readonly("effective_div", &RiemannPlan::effective_div)
      .def_property_readonly("compute_stream", [](const RiemannPlan& p) { return reinterpret_cast<uintptr_t>(p.compute_stream()); })
      .def_property_readonly("comm_stream", [](const RiemannPlan& p) { return reinterpret_cast<uintptr_t>(p.comm_stream()); })
      .def("run", &RiemannPlan::run, py::call_guard<py::gil_scoped_release>())
      .def("capture_graphs", &RiemannPlan::capture_graphs, py::call_guard<py::gil_scoped_release>())
      .def("prepare_steps", &RiemannPlan::prepare_steps, py::arg("steps"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("graph_launches", &RiemannPlan::graph_launches)
      .def_property_readonly("direct_steps", &RiemannPlan::direct_steps)
      .def("launch_steps", &RiemannPlan::launch_steps, py::arg("steps"), py::arg("pipeline") = true,
           py::arg("graphs") = true, py::call_guard<py::gil_scoped_release>())
      .def("sync", &RiemannPlan::sync, py::call_guard<py::gil_scoped_release>())
      .def("run_steps", [](RiemannPlan& p, int steps, bool pipeline, bool graphs) {
             StepTiming t;
             {
               py::gil_scoped_release nogil;
               t = p.run_steps(steps, pipeline, graphs);
             }
             py::dict r;
             r["wall_s"] = t.wall_s;
             r["device_ms"] = t.device_ms;
             r["steps"] = t.steps;
             return r;
           }, py::arg("steps"), py::arg("pipeline") = true, py::arg("graphs") = true)
      .def("barrier", &RiemannPlan::barrier, py::call_guard<py::gil_scoped_release>())
      .def("time_one_shot", [](RiemannPlan& p, int reps, const std::string& mode, int warmup) {
             OneShotTiming t;
             {
               py::gil_scoped_release nogil;
               t = p.time_one_shot(reps, mode, warmup);
             }
             py::dict r;
             r["mode"] = t.mode;
             r["reps"] = t.reps;
             r["median_us"] = t.median_us;
             r["min_us"] = t.min_us;
             r["max_us"] = t.max_us;
             r["device_median_us"] = t.device_median_us;
             r["device_min_us"] = t.device_min_us;
             r["value"] = t.value;
             return r;
           }, py::arg("reps"), py::arg("mode") = "direct", py::arg("warmup") = 400)
      .def("diagnose_batch", [](RiemannPlan& p, int steps) {
             BatchDiag d;
             {
               py::gil_scoped_release nogil;
               d = p.diagnose_batch(steps);
             }
             py::dict r;
             r["steps"] = d.steps;
             r["compute_us"] = d.compute_us;
             r["close_us"] = d.close_us;
             r["allreduce_us"] = d.allreduce_us;
             r["copy_us"] = d.copy_us;
             r["tail_us"] = d.tail_us();
             r["boundary_us"] = d.boundary_us();
             r["marker_us"] = d.marker_us;
             r["device_us"] = d.device_us;
             r["staged_us"] = d.staged_us;
             r["wall_us"] = d.wall_us;
             return r;
           }, py::arg("steps"))
      .def("host_result", &RiemannPlan::host_result)
      .def_property_readonly("host_capacity", &RiemannPlan::host_capacity)
      .def_property_readonly("slots", &RiemannPlan::slots)
      .def_property_readonly("bucketed", &RiemannPlan::bucketed)
      .def_property_readonly("chained", &RiemannPlan::chained)
      .def_property_readonly("multistep", &RiemannPlan::multistep)
      .def_property_readonly("close_in_launch", &RiemannPlan::close_in_launch)
      .def_property_readonly("allreduce_to_host", &RiemannPlan::allreduce_to_host)
      .def_property_readonly("direct", &RiemannPlan::direct)
      .def_property_readonly("graph_nodes", &RiemannPlan::graph_nodes)
      .def_property_readonly("graphs_ready", &RiemannPlan::graphs_ready)
      .def_property_readonly("graph_error", &RiemannPlan::graph_error)
      .def_property_readonly("collective", &RiemannPlan::collective)
      .def("host_index_of", &RiemannPlan::host_index_of, py::arg("k"), py::arg("graphs"))
      .def("enqueue", [](const RiemannPlan& p, uintptr_t s, int slot, int hidx) { p.enqueue(stream(s), slot, hidx); })
      .def("device_result", [](const RiemannPlan& p, int slot) { return reinterpret_cast<uintptr_t>(p.device_result(slot)); });

  // ------------------------------------------------------------------ raw kernels
  m.def("launch_riemann_partials",
        [](int integrand, double a, double h, double off, uint64_t i_begin, uint64_t n,
           std::vector<double> coef, double p0, double p1, DType dtype, DivMode div, int grid,
           uintptr_t table, int table_n, uintptr_t partials, uintptr_t s) {
          const RiemannParams p = make_params(integrand, a, h, off, i_begin, n, coef, p0, p1);
          launch_riemann_partials(p, dtype, div, {grid, kRiemannBlock}, ptr<const double>(table),
                                  table_n, ptr<double>(partials), stream(s));
        });
  m.def("launch_riemann_fused",
        [](int integrand, double a, double h, double off, uint64_t i_begin, uint64_t n,
           std::vector<double> coef, double p0, double p1, DType dtype, DivMode div, int grid,
           uintptr_t table, int table_n, uintptr_t partials, uintptr_t ticket, double scale,
           uintptr_t out, uintptr_t s) {
          const RiemannParams p = make_params(integrand, a, h, off, i_begin, n, coef, p0, p1);
          launch_riemann_fused(p, dtype, div, {grid, kRiemannBlock}, ptr<const double>(table),
                               table_n, ptr<double>(partials), ptr<unsigned>(ticket), scale,
                               ptr<double>(out), stream(s));
        });
  m.def("launch_riemann_point_values",
        [](int integrand, double a, double h, double off, uint64_t i_begin, uint64_t n,
           std::vector<double> coef, double p0, double p1, DivMode div, uintptr_t table,
           int table_n, uintptr_t out, uintptr_t s) {
          const RiemannParams p = make_params(integrand, a, h, off, i_begin, n, coef, p0, p1);
          launch_riemann_point_values(p, div, ptr<const double>(table), table_n, ptr<double>(out),
                                      stream(s));
        });
  m.def("launch_pi4_recip_narrow", [](uintptr_t d, uint64_t n, uintptr_t out, uintptr_t s) {
    launch_pi4_recip_narrow(ptr<const double>(d), n, ptr<double>(out), stream(s));
  });
  m.def("launch_pi4_recip_narrow_f32", [](uintptr_t d, uint64_t n, uintptr_t out, uintptr_t s) {
    launch_pi4_recip_narrow_f32(ptr<const float>(d), n, ptr<float>(out), stream(s));
  });
  m.def("set_lds_poison", &set_lds_poison, py::arg("on"),
        "validation: staged-window kernels fill their LDS with NaN first (current device)");
  m.def("set_trig_library", &set_trig_library, py::arg("on"),
        "validation: kIeee sin/cos by ocml per sample (SinLib / TrainVelLib)");
  m.def("fast_trig_host", [](uintptr_t x, uint64_t n, int shift, uintptr_t val, uintptr_t ulp) {
    // the device's per-sample sin/cos (fast_trig.hpp, compiled for the host) and its error in
    // ulps against long double sinl/cosl; NaN value/ulp where the tile path declines
    const double* xs = reinterpret_cast<const double*>(x);
    double* v = reinterpret_cast<double*>(val);
    double* e = reinterpret_cast<double*>(ulp);
    for (uint64_t i = 0; i < n; ++i) {
      double out;
      if (!fast_trig_point(xs[i], shift, out)) {
        v[i] = e[i] = std::nan("");
        continue;
      }
      const long double ref = shift ? cosl(static_cast<long double>(xs[i]))
                                    : sinl(static_cast<long double>(xs[i]));
      const double rd = static_cast<double>(ref);
      const double sp = std::nextafter(std::fabs(rd), INFINITY) - std::fabs(rd);
      v[i] = out;
      e[i] = static_cast<double>((static_cast<long double>(out) - ref) / sp);
    }
  });
  m.def("set_pi4_library_division", &set_pi4_library_division,
        "validation: kIeee Pi4 launches use the full library division (bitwise the same sums)");
  m.def("riemann_block_ok", &riemann_block_ok);
  m.def("launch_finalize", [](uintptr_t partials, int n, double scale, uintptr_t out, uintptr_t s,
                              int block) {
    launch_finalize(ptr<const double>(partials), n, scale, ptr<double>(out), stream(s), block);
  }, py::arg("partials"), py::arg("n"), py::arg("scale"), py::arg("out"), py::arg("stream"),
     py::arg("block") = kRiemannBlock);
  m.def("default_riemann_grid", [](int cus, int waves) { return default_riemann_shape(cus, waves).grid; });
  m.def("default_reduce_grid", &default_reduce_grid);
  m.def("launch_sum_array", [](uintptr_t x, uint64_t n, double scale, uintptr_t partials, int grid,
                               uintptr_t out, uintptr_t s) {
    launch_sum_array(ptr<const double>(x), n, scale, ptr<double>(partials), grid, ptr<double>(out), stream(s));
  });
  m.def("launch_interp_fill", [](uintptr_t table, int tn, double dt, uint64_t i0, uint64_t n,
                                 uintptr_t y, uintptr_t s) {
    launch_interp_fill(ptr<const double>(table), tn, dt, i0, n, ptr<double>(y), stream(s));
  });
  m.def("scan_state_bytes", &scan_state_bytes);
  m.def("launch_inclusive_scan", [](uintptr_t in, uintptr_t out, uint64_t n, uintptr_t state,
                                    uintptr_t carry, uintptr_t s) {
    launch_inclusive_scan(ptr<const double>(in), ptr<double>(out), n, ptr<void>(state),
                          ptr<const double>(carry), stream(s));
  });
  m.def("launch_interp_scan", [](uintptr_t table, int tn, double dt, uint64_t i0, uint64_t n,
                                 uint64_t win_lo, uint64_t win_hi, uintptr_t out, uintptr_t state,
                                 uintptr_t carry, uintptr_t s) {
    launch_interp_scan_window(ptr<const double>(table), tn, dt, i0, n, win_lo, win_hi,
                              ptr<double>(out), ptr<void>(state), ptr<const double>(carry), stream(s));
  });
  m.def("scan_timeout_flag", [](uintptr_t state, uintptr_t s) { return scan_timeout_flag(ptr<const void>(state), stream(s)); });
  m.def("launch_add_carry", [](uintptr_t x, uint64_t n, uintptr_t carry, uintptr_t s) {
    launch_add_carry(ptr<double>(x), n, ptr<const double>(carry), stream(s));
  });
  m.def("table2d_grid", [](int nx, int ny, double X, double Y, int gx, int gy, int row0, int row1) {
    Table2DParams p{nullptr, nx, ny, X, Y, gx, gy, row0, row1};
    return table2d_grid(p);
  });
  m.def("table2d_path", [](int nx, int ny, double X, double Y, int gx, int gy, int row0, int row1) {
    Table2DParams p{nullptr, nx, ny, X, Y, gx, gy, row0, row1};
    return std::string(table2d_path(p));
  });
  m.def("table2d_shape_info", [](int nx, int ny, double X, double Y, int gx, int gy, int row0,
                                 int row1, int min_wg) {
    Table2DParams p{nullptr, nx, ny, X, Y, gx, gy, row0, row1, min_wg};
    const Table2DShapeInfo i = table2d_shape_info(p);
    py::dict d;
    d["stream"] = i.stream;
    d["rows_per_wave"] = i.rows_per_wave;
    d["tile_rows"] = i.tile_rows;
    d["tile_cols"] = i.tile_cols;
    d["grid"] = py::make_tuple(i.grid_x, i.grid_y);
    d["tile"] = i.tile;
    return d;
  }, py::arg("nx"), py::arg("ny"), py::arg("X"), py::arg("Y"), py::arg("gx"), py::arg("gy"),
     py::arg("row0"), py::arg("row1"), py::arg("min_wg") = 0);
  m.def("launch_table2d_partials", [](uintptr_t table, int nx, int ny, double X, double Y, int gx,
                                      int gy, int row0, int row1, uintptr_t partials, uintptr_t s) {
    Table2DParams p{ptr<const double>(table), nx, ny, X, Y, gx, gy, row0, row1};
    launch_table2d_partials(p, ptr<double>(partials), stream(s));
  });
  m.def("launch_table2d_fused", [](uintptr_t table, int nx, int ny, double X, double Y, int gx,
                                    int gy, int row0, int row1, uintptr_t partials,
                                    uintptr_t ticket, uintptr_t out, uintptr_t s) {
    Table2DParams p{ptr<const double>(table), nx, ny, X, Y, gx, gy, row0, row1};
    launch_table2d_fused(p, ptr<double>(partials), ptr<unsigned>(ticket), ptr<double>(out),
                         stream(s));
  });
  m.def("launch_table2d_chained", [](uintptr_t table, int nx, int ny, double X, double Y, int gx,
                                      int gy, int row0, int row1, uintptr_t partials,
                                      uintptr_t prev, uintptr_t prev_out, uintptr_t s) {
    Table2DParams p{ptr<const double>(table), nx, ny, X, Y, gx, gy, row0, row1};
    launch_table2d_chained(p, ptr<double>(partials), ptr<const double>(prev),
                           ptr<double>(prev_out), stream(s));
  });
  m.def("launch_table2d_finalize", [](uintptr_t partials, int n, uintptr_t out, uintptr_t s) {
    launch_table2d_finalize(ptr<const double>(partials), n, ptr<double>(out), stream(s));
  });
  m.def("launch_outer_product", [](uintptr_t v, int n, uintptr_t t, uintptr_t s) {
    launch_outer_product(ptr<const double>(v), n, ptr<double>(t), stream(s));
  });
  m.def("selftest_wave_ops", [](uintptr_t in, uint64_t n, bool f32, uintptr_t sums, uintptr_t scan, uintptr_t s) {
    selftest_wave_ops(ptr<const void>(in), n, f32, ptr<void>(sums), ptr<void>(scan), stream(s));
  });
  m.def("selftest_block_ops", [](uintptr_t in, uint64_t n, int block, bool f32, uintptr_t sums,
                                 uintptr_t scan, uintptr_t s) {
    selftest_block_ops(ptr<const void>(in), n, block, f32, ptr<void>(sums), ptr<void>(scan), stream(s));
  });

  // ------------------------------------------------------------------ train scan pipeline
  py::class_<TrainScanConfig>(m, "TrainScanConfig")
      .def(py::init<>())
      .def_readwrite("steps_per_sec", &TrainScanConfig::steps_per_sec)
      .def_readwrite("seconds", &TrainScanConfig::seconds)
      .def_readwrite("parity", &TrainScanConfig::parity)
      .def_readwrite("replicate", &TrainScanConfig::replicate)
      .def_readwrite("phase2", &TrainScanConfig::phase2)
      .def_readwrite("table", &TrainScanConfig::table)
      .def_property("algo", [](const TrainScanConfig& c) { return scan_algo_name(c.algo); },
                    [](TrainScanConfig& c, const std::string& s) {
                      c.algo = scan_algo_of(s);
                    });
  m.def("trainscan_workspace_bytes", &trainscan_workspace_bytes);
  // the --replicate fingerprint (host code): FNV-1a over the fp64 bits, compensated sum,
  // elements at 0, n/4, n/2, 3n/4, n-1
  m.def("replica_digest", [](const std::vector<double>& v) {
    const ReplicaDigest d = digest_table(v.data(), v.size());
    py::dict r;
    r["hash"] = d.hash;
    r["n"] = d.n;
    r["sum"] = d.sum;
    r["at"] = std::vector<double>(d.at, d.at + 5);
    return r;
  });

  // ------------------------------------------------------------------ 2-D field plan
  py::class_<Table2DPlan>(m, "Table2DPlan")
      .def(py::init([](int grid, double extent, int device, const Comm* comm, bool bucket,
                       bool chain, int step_streams, int slice_rank, int slice_world,
                       bool multistep, int phases, int min_wg, int graph_steps,
                       bool force_collective) {
             Table2DConfig c;
             c.force_collective = force_collective;
             c.graph_steps = graph_steps;
             c.phases = phases;
             c.min_wg = min_wg;
             c.grid = grid;
             c.extent = extent;
             c.bucket = bucket;
             c.chain = chain;
             c.step_streams = step_streams;
             c.multistep = multistep;
             c.rank = slice_rank;   // without a communicator: that rank's rows only
             c.world = slice_world;
             return new Table2DPlan(c, device, comm);
           }),
           py::arg("grid") = 4096, py::arg("extent") = 1800.0, py::arg("device") = 0,
           py::arg("comm") = nullptr, py::arg("bucket") = true, py::arg("chain") = true,
           py::arg("step_streams") = 0, py::arg("slice_rank") = 0, py::arg("slice_world") = 1,
           py::arg("multistep") = true, py::arg("phases") = 0, py::arg("min_wg") = 0,
           py::arg("graph_steps") = 0, py::arg("force_collective") = false,
           py::keep_alive<1, 5>())
      .def_property_readonly("phases", &Table2DPlan::phases)
      .def_property_readonly("min_wg", &Table2DPlan::min_wg)
      .def_property_readonly("workgroups", &Table2DPlan::workgroups)
      .def_property_readonly("resident_per_cu", &Table2DPlan::resident_per_cu)
      .def_property_readonly("step_streams",
                             [](const Table2DPlan& p) { return p.step_streams(); })
      .def_property_readonly("multistep", &Table2DPlan::multistep)
      .def("run", &Table2DPlan::run, py::call_guard<py::gil_scoped_release>())
      .def("time", &Table2DPlan::time, py::arg("iters"), py::arg("graphs") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("last_result", &Table2DPlan::last_result)
      .def_property_readonly("bucketed", &Table2DPlan::bucketed)
      .def_property_readonly("chained", &Table2DPlan::chained)
      .def_property_readonly("collective", &Table2DPlan::collective)
      .def_property_readonly("graph_steps", &Table2DPlan::graph_steps)
      .def_property_readonly("row0", &Table2DPlan::row0)
      .def_property_readonly("row1", &Table2DPlan::row1);
  m.def("table2d_oracle", &table2d_oracle, py::arg("grid"), py::arg("extent") = 1800.0);
  m.def("table2d_auto_graph_steps", &table2d_auto_graph_steps, py::arg("grid"),
        py::arg("extent") = 1800.0, py::arg("world") = 1);
  m.def("launch_trainscan", [](uintptr_t table, int tn, double dt, uint64_t i0, uint64_t n,
                               uint64_t win_lo, uint64_t win_hi, uintptr_t ws, uintptr_t totals,
                               uintptr_t carries, uintptr_t vel, uintptr_t pos, uintptr_t s) {
    TrainScanKernelParams p{ptr<const double>(table), tn, dt, i0, n, win_lo, win_hi};
    launch_trainscan_local(p, ptr<void>(ws), ptr<double>(totals), stream(s));
    launch_trainscan_write(p, ptr<const void>(ws), ptr<const double>(carries), ptr<double>(vel),
                           ptr<double>(pos), stream(s));
  });
  m.def("launch_trainscan_onepass", [](uintptr_t table, int tn, double dt, uint64_t i0,
                                       uint64_t n, uint64_t win_lo, uint64_t win_hi, uintptr_t ws,
                                       uintptr_t totals, uintptr_t vel, uintptr_t pos,
                                       uintptr_t s) {
    TrainScanKernelParams p{ptr<const double>(table), tn, dt, i0, n, win_lo, win_hi};
    launch_trainscan_onepass(p, ptr<void>(ws), ptr<double>(vel), ptr<double>(pos),
                             ptr<double>(totals), stream(s));
  });
  m.def("trainscan_onepass_timeout", [](uintptr_t ws, uintptr_t s) {
    return trainscan_onepass_timeout(ptr<const void>(ws), stream(s));
  });
  py::class_<TrainScan>(m, "TrainScan")
      .def(py::init<const TrainScanConfig&, int, const Comm*>(), py::arg("config"),
           py::arg("device"), py::arg("comm") = nullptr, py::keep_alive<1, 4>())
      .def("run", [](TrainScan& t) {
        TrainScanResult r;
        {
          py::gil_scoped_release nogil;
          r = t.run();
        }
        py::dict d;
        d["distance"] = r.distance;
        d["sum_of_sums"] = r.sum_of_sums;
        d["distance_scan"] = r.distance_scan;
        d["device_ms"] = r.device_ms;
        d["timeout"] = r.timeout;
        return d;
      })
      .def_property_readonly("local_begin", &TrainScan::local_begin)
      .def_property_readonly("algo", [](const TrainScan& t) { return scan_algo_name(t.algo()); })
      .def_property_readonly("local_count", &TrainScan::local_count)
      .def("velocity_ptr", [](const TrainScan& t) { return reinterpret_cast<uintptr_t>(t.velocity()); })
      .def("position_ptr", [](const TrainScan& t) { return reinterpret_cast<uintptr_t>(t.position()); })
      .def("replicated_ptr", [](const TrainScan& t) { return reinterpret_cast<uintptr_t>(t.replicated()); })
      .def_property_readonly("total", &TrainScan::total);

  // ------------------------------------------------------------------ runtime integrands
  m.def("expr_source", &expr_source, "kernel source generated for an expression over x");
  m.def("expr_compile", [](const std::string& e) {
          std::string code;
          {
            py::gil_scoped_release nogil;
            code = expr_compile(e);
          }
          return py::bytes(code);
        },
        "compile an expression for gfx950 with hipRTC (no device needed); the code object");
  py::class_<ExprIntegrator>(m, "ExprIntegrator",
                             "f(x) given as an expression, compiled with hipRTC for gfx950")
      .def(py::init<const std::string&, int, int>(), py::arg("expr"), py::arg("device") = 0,
           py::arg("grid") = 2048)
      .def("integrate", &ExprIntegrator::integrate, py::arg("a"), py::arg("b"), py::arg("n"),
           py::arg("rule"), py::arg("begin"), py::arg("count"), py::arg("scale") = 1.0,
           py::arg("comm") = nullptr, py::call_guard<py::gil_scoped_release>())
      .def("time",
           [](ExprIntegrator& e, double a, double b, uint64_t n, Rule rule, uint64_t begin,
              uint64_t count, int iters) { return e.time(a, b, n, rule, begin, count, iters); },
           py::arg("a"), py::arg("b"), py::arg("n"), py::arg("rule"), py::arg("begin"),
           py::arg("count"), py::arg("iters"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("expression", &ExprIntegrator::expression);

  // ------------------------------------------------------------------ host (CPU) engine
  m.def("host_isa", &host_isa, "vector ISA the host kernels dispatch to: avx512|avx2|base");
  py::class_<HostPool>(m, "HostPool", "persistent host worker threads (0 = one per core)")
      .def(py::init<int>(), py::arg("threads") = 0)
      .def_property_readonly("threads", &HostPool::threads)
      .def_static("default_threads", &HostPool::default_threads);
  m.def("host_riemann", &host_riemann, py::arg("config"), py::arg("begin"), py::arg("count"),
        py::arg("pool"), py::call_guard<py::gil_scoped_release>(),
        "h * scale * sum of f over samples [begin, begin + count), per-sample fp64 on threads");
  py::class_<HostExpr>(m, "HostExpr", "f(x) as an expression, compiled for the host cores")
      .def(py::init<const std::string&>(), py::arg("expr"),
           py::call_guard<py::gil_scoped_release>())
      .def("integrate", &HostExpr::integrate, py::arg("a"), py::arg("b"), py::arg("n"),
           py::arg("rule"), py::arg("begin"), py::arg("count"), py::arg("pool"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("expression", &HostExpr::expression);
  m.def("host_riemann_mpi_parity", &host_riemann_mpi_parity, py::arg("comm_size"), py::arg("n"),
        py::arg("range"), py::arg("pool"), py::call_guard<py::gil_scoped_release>(),
        "the reference's mpirun -np P ./riemann, bit for bit, with its P-1 workers on threads");
  py::class_<HostComm>(m, "HostComm", "host collectives between processes (TCP star via rank 0)")
      .def(py::init<const std::string&, int, int, int, double>(), py::arg("addr"),
           py::arg("port"), py::arg("rank"), py::arg("world"), py::arg("timeout_s") = 120.0,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rank", &HostComm::rank)
      .def_property_readonly("world", &HostComm::world)
      .def("allreduce_sum", [](HostComm& c, std::vector<double> v) {
             py::gil_scoped_release nogil;
             c.allreduce_sum(v.data(), v.size());
             return v;
           })
      .def("allgather", [](HostComm& c, std::vector<double> v) {
             std::vector<double> out(v.size() * c.world());
             py::gil_scoped_release nogil;
             c.allgather(v.data(), out.data(), v.size());
             return out;
           })
      .def("broadcast", [](HostComm& c, std::vector<double> v, int root) {
             py::gil_scoped_release nogil;
             c.broadcast(v.data(), v.size(), root);
             return v;
           })
      .def("barrier", &HostComm::barrier, py::call_guard<py::gil_scoped_release>());
  m.def("host_trainscan", [](int sps, int seconds, HostPool& pool, HostComm* comm, bool keep,
                             std::vector<double> table) {
          HostScanConfig c;
          c.steps_per_sec = sps;
          c.seconds = seconds;
          c.keep = keep;
          c.table = std::move(table);
          std::vector<double> vel, pos;
          HostScanResult r;
          {
            py::gil_scoped_release nogil;
            r = host_trainscan(c, pool, comm, keep ? &vel : nullptr, keep ? &pos : nullptr);
          }
          py::dict d;
          d["distance"] = r.distance;
          d["sum_of_sums"] = r.sum_of_sums;
          d["seconds"] = r.seconds;
          d["begin"] = r.begin;
          d["count"] = r.count;
          if (keep) {
            d["velocity"] = vel;
            d["position"] = pos;
          }
          return d;
        },
        py::arg("steps_per_sec") = 10000, py::arg("seconds") = 1800, py::arg("pool"),
        py::arg("comm") = nullptr, py::arg("keep") = false,
        py::arg("table") = std::vector<double>{});

  // ------------------------------------------------------------------ oracle
  py::module_ o = m.def_submodule("oracle", "host oracles, generated fixtures, parity emulation");
  o.def("profile_table", &oracle::profile_table);
  o.def("generated_profile_table", &oracle::generated_profile_table);
  o.def("faccel_ref", [](double t) { return oracle::faccel_ref(oracle::profile_table(), t); });
  o.def("interp", [](double t) { return oracle::interp(oracle::profile_table(), t); });
  o.def("profile_exact_integral", &oracle::profile_exact_integral);
  o.def("load_profile", &oracle::load_profile, py::arg("path"),
        "a velocity profile (CSV/text numbers, 1 s spacing)");
  o.def("table_integral", &oracle::table_integral, py::arg("table"), py::arg("a"), py::arg("b"),
        "exact integral of the table's piecewise-linear interpolant over [a, b]");
  o.def("analytic", &oracle::analytic, py::arg("integrand"), py::arg("a"), py::arg("b"),
        py::arg("coef") = std::vector<double>{}, py::arg("p0") = 0.0, py::arg("p1") = 0.0);
  o.def("riemann_serial", [](Integrand f, double a, double b, uint64_t n, Rule r,
                             std::vector<double> coef, double p0, double p1) {
    py::gil_scoped_release nogil;
    return static_cast<double>(oracle::riemann_serial(f, a, b, n, r, coef, p0, p1));
  }, py::arg("integrand"), py::arg("a"), py::arg("b"), py::arg("n"), py::arg("rule"),
     py::arg("coef") = std::vector<double>{}, py::arg("p0") = 0.0, py::arg("p1") = 0.0);
  o.def("riemann_mpi_parity", &oracle::riemann_mpi_parity, py::arg("comm_size"), py::arg("n"),
        py::arg("range") = 3.14159265358979323846, py::call_guard<py::gil_scoped_release>());
  o.def("cintegrate_parity", &oracle::cintegrate_parity, py::call_guard<py::gil_scoped_release>());
  o.def("trainscan_parity", [](int p) {
    oracle::TrainScanParity r;
    {
      py::gil_scoped_release nogil;
      r = oracle::trainscan_parity(p);
    }
    return py::make_tuple(r.distance, r.sum_of_sums);
  });
  o.def("train_distance", &oracle::train_distance);
  o.attr("TRAIN_TS") = oracle::kTrainTs;
  o.attr("TRAIN_VS") = oracle::kTrainVs;
  o.attr("TRAIN_AS") = oracle::kTrainAs;
  o.attr("STEPS_PER_SEC") = oracle::kStepsPerSec;
  o.attr("PROFILE_SECONDS") = oracle::kProfileSeconds;
}
