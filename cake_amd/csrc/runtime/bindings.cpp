// pybind11 module `_cake_runtime`: the native host runtime exposed to Python.
// Blocking socket calls release the GIL so worker connection threads run in
// parallel with model compute.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "json.h"
#include "net.h"
#include "proto.h"
#include "safetensors.h"
#include "server.h"
#include "topology.h"

namespace py = pybind11;
using namespace cake;

namespace {

py::list topo_to_py(const Topology& t) {
  py::list out;
  for (const auto& n : t.nodes) {
    py::dict d;
    d["name"] = n.name;
    d["host"] = n.host;
    d["description"] = n.has_description ? py::object(py::str(n.description)) : py::none();
    d["layers"] = n.layers;
    out.append(d);
  }
  return out;
}

Message msg_from_py(const py::dict& d, py::object data, py::buffer_info* keep) {
  Message m;
  m.type = (MsgType)d["type"].cast<uint32_t>();
  if (d.contains("layer_name")) m.layer_name = d["layer_name"].cast<std::string>();
  if (d.contains("index_pos")) m.index_pos = d["index_pos"].cast<uint64_t>();
  if (d.contains("block_idx")) m.block_idx = d["block_idx"].cast<uint64_t>();
  if (d.contains("error")) m.error = d["error"].cast<std::string>();
  if (d.contains("session")) m.session = d["session"].cast<uint64_t>();
  if (d.contains("batch"))
    for (auto item : d["batch"].cast<py::list>()) {
      auto t = item.cast<py::tuple>();
      m.batch.push_back({t[0].cast<std::string>(), t[1].cast<uint64_t>(), t[2].cast<uint64_t>()});
    }
  if (d.contains("info")) {
    auto i = d["info"].cast<py::dict>();
    m.info.version = i["version"].cast<std::string>();
    m.info.dtype = i["dtype"].cast<std::string>();
    m.info.os = i["os"].cast<std::string>();
    m.info.arch = i["arch"].cast<std::string>();
    m.info.device = i["device"].cast<std::string>();
    m.info.device_idx = i["device_idx"].cast<uint64_t>();
    m.info.latency_lo = i["latency"].cast<uint64_t>();
  }
  if (d.contains("dtype")) m.x.dtype = d["dtype"].cast<std::string>();
  if (d.contains("shape")) m.x.shape = d["shape"].cast<std::vector<uint64_t>>();
  if (!data.is_none()) {
    *keep = data.cast<py::buffer>().request();
    m.x.data = static_cast<const uint8_t*>(keep->ptr);
    m.x.nbytes = (uint64_t)(keep->size * keep->itemsize);
  }
  return m;
}

py::dict msg_to_py(const Message& m, const uint8_t* body_base) {
  py::dict d;
  d["type"] = (uint32_t)m.type;
  switch (m.type) {
    case MsgType::WorkerInfo: {
      py::dict i;
      i["version"] = m.info.version;
      i["dtype"] = m.info.dtype;
      i["os"] = m.info.os;
      i["arch"] = m.info.arch;
      i["device"] = m.info.device;
      i["device_idx"] = m.info.device_idx;
      i["latency"] = m.info.latency_lo;
      d["info"] = i;
      break;
    }
    case MsgType::SingleOp:
      d["layer_name"] = m.layer_name;
      d["index_pos"] = m.index_pos;
      d["block_idx"] = m.block_idx;
      break;
    case MsgType::Batch: {
      py::list b;
      for (const auto& it : m.batch) b.append(py::make_tuple(it.layer_name, it.index_pos, it.block_idx));
      d["batch"] = b;
      break;
    }
    case MsgType::Error: d["error"] = m.error; break;
    case MsgType::Reset: d["session"] = m.session; break;
    default: break;
  }
  if (m.type == MsgType::SingleOp || m.type == MsgType::Batch || m.type == MsgType::Tensor) {
    d["dtype"] = m.x.dtype;
    d["shape"] = m.x.shape;
    d["offset"] = (uint64_t)(m.x.data - body_base);
    d["nbytes"] = m.x.nbytes;
  }
  return d;
}

}  // namespace

PYBIND11_MODULE(_cake_runtime, mod) {
  mod.doc() = "cake_amd native host runtime (topology, wire codec, TCP, safetensors)";

  // ---------------------------------------------------------------- topology
  mod.def("parse_topology", [](const std::string& text, bool text_model) {
    return topo_to_py(Topology::parse(text, text_model));
  }, py::arg("text"), py::arg("text_model") = true);
  mod.def("load_topology", [](const std::string& path, bool text_model) {
    return topo_to_py(Topology::from_path(path, text_model));
  }, py::arg("path"), py::arg("text_model") = true);
  mod.def("expand_layer_range", &expand_layer_range);

  // ---------------------------------------------------------------- protocol
  mod.attr("PROTO_MAGIC") = kProtoMagic;
  mod.attr("MESSAGE_MAX_SIZE") = kMaxMessageSize;
  mod.def("encode_message", [](const py::dict& d, py::object data) {
    py::buffer_info keep;
    Message m = msg_from_py(d, data, &keep);
    std::string body = encode_body(m);
    return py::bytes(body);
  }, py::arg("msg"), py::arg("data") = py::none());
  mod.def("decode_message", [](py::bytes body) {
    std::string_view v(body);
    Message m = decode_body(reinterpret_cast<const uint8_t*>(v.data()), v.size());
    return msg_to_py(m, reinterpret_cast<const uint8_t*>(v.data()));
  });
  mod.def("encode_header", [](uint32_t n) {
    uint8_t h[8];
    encode_header(n, h);
    return py::bytes(reinterpret_cast<const char*>(h), 8);
  });
  mod.def("decode_header", [](py::bytes b) {
    std::string s = b;
    if (s.size() != 8) throw std::runtime_error("header must be 8 bytes");
    return decode_header(reinterpret_cast<const uint8_t*>(s.data()));
  });

  // ---------------------------------------------------------------- sockets
  mod.def("tcp_listen", [](const std::string& host, int port) {
    py::gil_scoped_release nogil;
    return tcp_listen(host, port);
  });
  mod.def("tcp_accept", [](int fd) {
    std::string peer;
    int c;
    {
      py::gil_scoped_release nogil;
      c = tcp_accept(fd, &peer);
    }
    return py::make_tuple(c, peer);
  });
  mod.def("tcp_connect", [](const std::string& host, int port, double timeout) {
    py::gil_scoped_release nogil;
    return tcp_connect(host, port, timeout);
  }, py::arg("host"), py::arg("port"), py::arg("timeout") = 10.0);
  mod.def("tcp_set_timeout", &tcp_set_timeout);
  mod.def("tcp_close", &tcp_close);
  mod.def("tcp_local_port", &tcp_local_port);
  mod.def("send_message", [](int fd, const py::dict& d, py::object data) {
    py::buffer_info keep;
    Message m = msg_from_py(d, data, &keep);
    std::string body = encode_body(m);
    py::gil_scoped_release nogil;
    return send_frame(fd, reinterpret_cast<const uint8_t*>(body.data()), (uint32_t)body.size());
  }, py::arg("fd"), py::arg("msg"), py::arg("data") = py::none());
  mod.def("recv_message", [](int fd) {
    std::string body;
    {
      py::gil_scoped_release nogil;
      body = recv_frame(fd);
    }
    Message m = decode_body(reinterpret_cast<const uint8_t*>(body.data()), body.size());
    py::dict d = msg_to_py(m, reinterpret_cast<const uint8_t*>(body.data()));
    const uint64_t n = body.size();
    return py::make_tuple(d, py::bytes(body), n + 8);
  });

  // ---------------------------------------------------------------- safetensors
  py::class_<SafeTensorsFile>(mod, "SafeTensorsFile")
      .def(py::init<const std::string&>())
      .def("names", &SafeTensorsFile::names)
      .def("metadata", &SafeTensorsFile::metadata)
      .def("__contains__", &SafeTensorsFile::has)
      .def("info", [](const SafeTensorsFile& f, const std::string& n) {
        const TensorView& v = f.tensor(n);
        py::dict d;
        d["dtype"] = v.dtype;
        d["shape"] = v.shape;
        d["offset"] = v.offset;
        d["nbytes"] = v.nbytes;
        return d;
      })
      .def("buffer", [](const SafeTensorsFile& f) {
        return py::memoryview::from_memory(const_cast<uint8_t*>(f.base()), (ssize_t)f.size(), /*readonly=*/true);
      }, py::keep_alive<0, 1>());
  mod.def("write_safetensors", [](const std::string& path, const py::list& tensors,
                                  const std::map<std::string, std::string>& metadata) {
    std::vector<TensorToWrite> out;
    std::vector<py::buffer_info> keep;
    keep.reserve(tensors.size());
    for (auto item : tensors) {
      auto t = item.cast<py::tuple>();
      keep.push_back(t[3].cast<py::buffer>().request());
      const auto& b = keep.back();
      out.push_back({t[0].cast<std::string>(), t[1].cast<std::string>(),
                     t[2].cast<std::vector<uint64_t>>(), static_cast<const uint8_t*>(b.ptr),
                     (uint64_t)(b.size * b.itemsize)});
    }
    py::gil_scoped_release nogil;
    write_safetensors(path, out, metadata);
  }, py::arg("path"), py::arg("tensors"), py::arg("metadata") = std::map<std::string, std::string>{});
  mod.def("load_weight_map", &load_weight_map);

  // ---------------------------------------------------------------- worker server
  py::class_<WorkerServer>(mod, "WorkerServer")
      .def(py::init([](const std::string& host, int port, const py::dict& i, const std::string& name) {
             WorkerInfo info;
             info.version = i["version"].cast<std::string>();
             info.dtype = i["dtype"].cast<std::string>();
             info.os = i["os"].cast<std::string>();
             info.arch = i["arch"].cast<std::string>();
             info.device = i["device"].cast<std::string>();
             info.device_idx = i["device_idx"].cast<uint64_t>();
             py::gil_scoped_release nogil;
             return new WorkerServer(host, port, info, name);
           }),
           py::arg("host"), py::arg("port"), py::arg("info"), py::arg("name"))
      .def_property_readonly("port", &WorkerServer::port)
      .def("serve", [](WorkerServer& s) {
        py::gil_scoped_release nogil;
        s.serve();
      })
      .def("stop", &WorkerServer::stop)
      .def("set_drop_after", &WorkerServer::set_drop_after)
      .def("set_stats_every", &WorkerServer::set_stats_every)
      .def("set_compute", [](WorkerServer& s, py::function fn) {
        // fn(session, ops[(name, pos, idx)], dtype, shape, memoryview) -> (dtype, shape, data)
        // data: bytes or any contiguous buffer (copied once into the reply)
        auto holder = std::make_shared<py::function>(std::move(fn));
        s.set_compute([holder](uint64_t session, const std::vector<BatchItem>& ops,
                               const RawTensor& x) -> OpResult {
          py::gil_scoped_acquire gil;
          OpResult r;
          try {
            py::list pops;
            for (const auto& o : ops) pops.append(py::make_tuple(o.layer_name, o.index_pos, o.block_idx));
            auto mv = py::memoryview::from_memory(const_cast<uint8_t*>(x.data), (ssize_t)x.nbytes, true);
            py::tuple out = (*holder)(session, pops, x.dtype, x.shape, mv);
            r.dtype = out[0].cast<std::string>();
            r.shape = out[1].cast<std::vector<uint64_t>>();
            py::object d = out[2];
            if (py::isinstance<py::bytes>(d)) {
              r.data = d.cast<std::string>();
            } else {
              py::buffer_info bi = d.cast<py::buffer>().request();
              r.data.assign(static_cast<const char*>(bi.ptr), (size_t)(bi.size * bi.itemsize));
            }
          } catch (py::error_already_set& e) {
            r.error = e.what();
          }
          return r;
        });
      })
      .def("set_reset", [](WorkerServer& s, py::function fn) {
        auto holder = std::make_shared<py::function>(std::move(fn));
        s.set_reset([holder](uint64_t session) { py::gil_scoped_acquire g; (*holder)(session); });
      })
      .def("set_drop", [](WorkerServer& s, py::function fn) {
        auto holder = std::make_shared<py::function>(std::move(fn));
        s.set_drop([holder](uint64_t session) { py::gil_scoped_acquire g; (*holder)(session); });
      })
      .def("set_log", [](WorkerServer& s, py::function fn) {
        auto holder = std::make_shared<py::function>(std::move(fn));
        s.set_log([holder](const std::string& m) { py::gil_scoped_acquire g; (*holder)(m); });
      })
      .def("stats", [](const WorkerServer& s) {
        const ServerStats& st = s.stats();
        py::dict d;
        d["connections"] = st.connections.load();
        d["messages"] = st.messages.load();
        d["ops"] = st.ops.load();
        d["bytes_in"] = st.bytes_in.load();
        d["bytes_out"] = st.bytes_out.load();
        d["errors"] = st.errors.load();
        return d;
      });
  mod.def("json_roundtrip", [](const std::string& s, int indent) { return Json::parse(s).dump(indent); },
          py::arg("text"), py::arg("indent") = -1);
}
