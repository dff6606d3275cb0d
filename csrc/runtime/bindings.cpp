// Python bindings of the native runtime core (module `moose_amd._native._moosert`).
//
// Parity: reference pymoose/src/bindings.rs exposes the Rust runtime to Python through
// PyO3; here pybind11 exposes the C++ parser, graph, networking and dataflow scheduler.
// The dataflow scheduler releases the GIL while it waits and re-acquires it only inside
// the per-operation callback, so operations whose kernels release the GIL (PyTorch ops,
// the native ring kernels, socket I/O) overlap across worker threads.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <climits>
#include <cmath>

#include "graph.h"
#include "net.h"
#include "scheduler.h"
#include "textual.h"

namespace py = pybind11;
using namespace moosert;

namespace {

AttrKind attr_kind(const std::string& k) {
  if (k == "int") return AttrKind::Int;
  if (k == "opt_int") return AttrKind::OptInt;
  if (k == "ints") return AttrKind::Ints;
  if (k == "opt_ints") return AttrKind::OptInts;
  if (k == "bool") return AttrKind::Bool;
  if (k == "str") return AttrKind::Str;
  if (k == "key") return AttrKind::Key;
  if (k == "const") return AttrKind::Const;
  if (k == "slice") return AttrKind::Slice;
  throw std::invalid_argument("unknown attribute kind " + k);
}

// Python int of arbitrary width from a decimal token (ring constants exceed 64 bits).
py::object int_of(std::string_view tok) {
  std::string s(tok);
  if (!s.empty() && s[0] == '+') s.erase(0, 1);
  PyObject* o = PyLong_FromString(s.c_str(), nullptr, 10);
  if (!o) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(o);
}

py::object num_of(const Num& n) {
  if (!n.is_float) return int_of(n.tok);
  std::string s(n.tok);
  if (s == "inf" || s == "+inf") return py::float_(HUGE_VAL);
  if (s == "-inf") return py::float_(-HUGE_VAL);
  if (s == "NaN") return py::float_(std::nan(""));
  return py::float_(std::strtod(s.c_str(), nullptr));
}

py::object opt_i64(int64_t v) { return v == INT64_MIN ? py::object(py::none()) : py::int_(v); }

// Attribute value -> Python.  Constants come back as ("const", kind, payload[, shape]);
// the Python side wraps them in IR `Constant`s (the numpy dtype choice lives there).
py::object value_to_py(const Value& v) {
  switch (v.tag) {
    case Value::None:
      return py::none();
    case Value::Int:
      return int_of(v.num.tok);
    case Value::Bool:
      return py::bool_(v.b);
    case Value::Str:
      return py::str(v.text);
    case Value::Ints: {
      py::list l;
      for (auto& n : v.nums) l.append(int_of(n.tok));
      return std::move(l);
    }
    case Value::Key:
      return py::bytes(reinterpret_cast<const char*>(v.bytes.data()), v.bytes.size());
    case Value::Const: {
      if (v.ckind == "HostString") return py::make_tuple("const", v.ckind, py::str(v.text));
      if (v.ckind == "HostSeed" || v.ckind == "HostPrfKey")
        return py::make_tuple(
            "const", v.ckind,
            py::bytes(reinterpret_cast<const char*>(v.bytes.data()), v.bytes.size()));
      py::list flat;
      for (auto& n : v.nums) flat.append(num_of(n));
      if (v.const_is_tensor) return py::make_tuple("const", v.ckind, flat, py::cast(v.shape));
      return py::make_tuple("const", v.ckind, flat);
    }
    case Value::Slice: {
      py::list out;
      for (auto& s : v.slices) out.append(py::make_tuple(s[0], opt_i64(s[1]), opt_i64(s[2])));
      if (v.slice_list) return std::move(out);
      return out[0];
    }
  }
  return py::none();
}

py::tuple record_to_py(const OpRecord& r) {
  py::list attrs;
  for (auto& kv : r.attrs) attrs.append(py::make_tuple(kv.first, value_to_py(kv.second)));
  py::object sig = py::none();
  if (r.has_sig) {
    py::list args;
    for (auto a : r.sig_args) args.append(py::str(a.data(), a.size()));
    sig = py::make_tuple(args, py::str(r.sig_ret.data(), r.sig_ret.size()), r.variadic);
  }
  py::list inputs;
  for (auto i : r.inputs) inputs.append(py::str(i.data(), i.size()));
  py::list owners;
  for (auto o : r.owners) owners.append(py::str(o.data(), o.size()));
  return py::make_tuple(py::str(r.name.data(), r.name.size()), r.kind, attrs, sig,
                        r.sig_ret_default, inputs, py::str(r.plc_kind.data(), r.plc_kind.size()),
                        owners);
}

std::shared_ptr<Schema> make_schema(const py::dict& ops, const py::dict& aliases,
                                    const py::dict& default_return) {
  auto s = std::make_shared<Schema>();
  for (auto kv : ops) {
    std::vector<std::pair<std::string, AttrKind>> attrs;
    for (auto a : kv.second.cast<py::sequence>()) {
      auto t = a.cast<py::sequence>();
      attrs.emplace_back(t[0].cast<std::string>(), attr_kind(t[1].cast<std::string>()));
    }
    s->ops.emplace(kv.first.cast<std::string>(), std::move(attrs));
  }
  for (auto kv : aliases)
    s->aliases.emplace(kv.first.cast<std::string>(), kv.second.cast<std::string>());
  for (auto kv : default_return)
    s->default_return.emplace(kv.first.cast<std::string>(), kv.second.cast<std::string>());
  return s;
}

py::dict stats_to_py(const RunStats& st) {
  py::dict d;
  d["ops_run"] = st.ops_run;
  d["max_parallel"] = st.max_parallel;
  d["wall_s"] = st.wall_s;
  d["wait_recv_s"] = st.wait_recv_s;
  return d;
}

}  // namespace

PYBIND11_MODULE(_moosert, m) {
  m.doc() = "moose_amd native runtime core: parser, graph passes, networking, dataflow";

  py::register_exception<ParseError>(m, "NativeParseError", PyExc_ValueError);
  py::register_exception<GraphError>(m, "NativeGraphError", PyExc_ValueError);
  auto net_err = py::register_exception<NetError>(m, "NativeNetError", PyExc_RuntimeError);
  py::register_exception<NetTimeout>(m, "NativeNetTimeout", net_err.ptr());

  py::class_<Schema, std::shared_ptr<Schema>>(m, "Schema")
      .def(py::init(&make_schema), py::arg("ops"), py::arg("aliases"), py::arg("default_return"));

  m.def(
      "parse",
      [](const std::string& src, const Schema& schema, int threads) {
        std::vector<OpRecord> recs;
        {
          py::gil_scoped_release nogil;
          recs = parse_computation(src, schema, threads);
        }
        py::list out;
        for (auto& r : recs) out.append(record_to_py(r));
        return out;
      },
      py::arg("source"), py::arg("schema"), py::arg("threads") = 8,
      "Parse a textual computation into operation records.");

  py::class_<Graph, std::shared_ptr<Graph>>(m, "Graph")
      .def(py::init<std::vector<std::string>, const std::vector<std::vector<std::string>>&,
                    std::vector<std::string>, std::vector<std::string>, std::vector<std::string>>(),
           py::arg("names"), py::arg("inputs"), py::arg("kinds"), py::arg("rendezvous"),
           py::arg("hosts"))
      .def("__len__", &Graph::size)
      .def("toposort", &Graph::toposort)
      .def("prune", &Graph::prune)
      .def("first_out_of_order", &Graph::first_out_of_order)
      .def("last_use", &Graph::last_use)
      .def("levels", &Graph::levels)
      .def("comm_rounds", &Graph::comm_rounds)
      .def("op_histogram", &Graph::op_histogram)
      .def("out_degree_histogram", &Graph::out_degree_histogram)
      .def("preds", [](const Graph& g, int32_t i) { return g.preds().at(i); })
      .def("succs", [](const Graph& g, int32_t i) { return g.succs().at(i); });

  py::class_<Mailbox, std::shared_ptr<Mailbox>>(m, "Mailbox")
      .def(py::init<>())
      .def("put",
           [](Mailbox& mb, const std::string& key, const std::string& sender, py::bytes payload) {
             Message msg{sender, std::string(payload)};
             py::gil_scoped_release nogil;
             mb.put(key, std::move(msg));
           })
      .def("has", &Mailbox::has)
      .def(
          "take",
          [](Mailbox& mb, const std::string& key, double timeout_s) {
            Message msg;
            {
              py::gil_scoped_release nogil;
              msg = mb.take(key, timeout_s);
            }
            return py::make_tuple(msg.sender, py::bytes(msg.payload));
          },
          py::arg("key"), py::arg("timeout_s") = -1.0)
      .def("abort", &Mailbox::abort, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("aborted", &Mailbox::aborted)
      .def("pending", &Mailbox::pending)
      .def("pending_keys", &Mailbox::pending_keys);

  py::class_<TcpNetworking, std::shared_ptr<TcpNetworking>>(m, "TcpNetworking")
      .def(py::init([](std::string own, std::map<std::string, std::string> endpoints,
                       std::shared_ptr<Mailbox> mb, double initial_s, double multiplier,
                       double max_interval_s, double max_elapsed_s, std::string cert_file,
                       std::string key_file, std::string ca_file) {
             BackoffPolicy b{initial_s, multiplier, max_interval_s, max_elapsed_s};
             TlsConfig tls{std::move(cert_file), std::move(key_file), std::move(ca_file)};
             return std::make_shared<TcpNetworking>(std::move(own), std::move(endpoints),
                                                    std::move(mb), b, std::move(tls));
           }),
           py::arg("own"), py::arg("endpoints"), py::arg("mailbox"), py::arg("initial_s") = 0.05,
           py::arg("multiplier") = 1.1, py::arg("max_interval_s") = 5.0,
           py::arg("max_elapsed_s") = 300.0, py::arg("cert_file") = "",
           py::arg("key_file") = "", py::arg("ca_file") = "")
      .def("start", &TcpNetworking::start, py::call_guard<py::gil_scoped_release>())
      .def("send",
           [](TcpNetworking& t, const std::string& receiver, const std::string& key,
              py::bytes payload) {
             std::string p(payload);
             py::gil_scoped_release nogil;
             t.send(receiver, key, std::move(p));
           })
      .def("flush", &TcpNetworking::flush, py::arg("timeout_s") = 300.0,
           py::call_guard<py::gil_scoped_release>())
      .def("close", &TcpNetworking::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &TcpNetworking::port)
      .def("stats", [](TcpNetworking& t) {
        py::dict d;
        for (auto& kv : t.stats()) {
          py::dict s;
          s["bytes_sent"] = kv.second.bytes_sent;
          s["bytes_recv"] = kv.second.bytes_recv;
          s["msgs_sent"] = kv.second.msgs_sent;
          s["msgs_recv"] = kv.second.msgs_recv;
          d[py::str(kv.first)] = s;
        }
        return d;
      });

  py::class_<Dataflow>(m, "Dataflow")
      .def(py::init<const Graph&, std::vector<int32_t>, std::vector<std::string>,
                    std::shared_ptr<Mailbox>>(),
           py::arg("graph"), py::arg("ops"), py::arg("wait_keys"), py::arg("mailbox") = nullptr,
           py::keep_alive<1, 2>())
      .def(
          "run",
          [](Dataflow& df, py::function cb, int workers, double timeout_s) {
            // Worker threads call back into Python holding the GIL only for the call; a
            // Python exception travels as error_already_set and is re-raised here.
            std::function<void(int32_t)> f = [&cb](int32_t i) {
              py::gil_scoped_acquire gil;
              cb(i);
            };
            RunStats st;
            {
              py::gil_scoped_release nogil;
              st = df.run(f, workers, timeout_s);
            }
            return stats_to_py(st);
          },
          py::arg("callback"), py::arg("workers") = 4, py::arg("timeout_s") = -1.0);
}
