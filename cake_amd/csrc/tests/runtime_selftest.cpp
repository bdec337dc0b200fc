// Native self-test of the C++ runtime (no GPU): JSON, topology, wire codec,
// safetensors, framed TCP and the multi-threaded WorkerServer.
//
// Built three ways by scripts/sanitize_runtime.sh / tests/test_sanitizers_cpu.py:
// plain, -fsanitize=address,undefined and -fsanitize=thread (host code only —
// ASan/UBSan for the host runtime, TSan for the worker/transport
// threads).  The server test drives several concurrent client connections,
// the stop() path while connections are open, fault injection (drop after N
// ops) and error replies, which is where data races would show.
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/json.h"
#include "../runtime/net.h"
#include "../runtime/proto.h"
#include "../runtime/safetensors.h"
#include "../runtime/server.h"
#include "../runtime/topology.h"

using namespace cake;

static int g_fail = 0;
#define CHECK(c)                                                             \
  do {                                                                       \
    if (!(c)) {                                                              \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)

static void test_topology() {
  const char* y =
      "# comment\n"
      "w0:\n  host: '10.0.0.1:10128'\n  description: first\n  layers:\n"
      "    - model.layers.0-3\n    - lm_head\n"
      "w1:\n  host: 10.0.0.2:10128\n  layers: [model.layers.4, model.layers.5-6]\n";
  Topology t = Topology::parse(y, true);
  CHECK(t.nodes.size() == 2);
  CHECK(t.nodes[0].layers.size() == 5);
  CHECK(t.node_for_layer("model.layers.2") == &t.nodes[0]);
  CHECK(t.node_for_layer("model.layers.6") == &t.nodes[1]);
  CHECK(t.node_for_layer("model.layers.7") == nullptr);
  CHECK(t.nodes[0].is_text_model_layer_owner("model.layers.3.mlp.up_proj.weight"));
  CHECK(!t.nodes[0].is_text_model_layer_owner("model.layers.30.mlp.up_proj.weight"));
  bool threw = false;
  try {
    expand_layer_range("model.layers.5-5");
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
  Topology back = Topology::parse(t.to_yaml(), true);
  CHECK(back.nodes.size() == 2 && back.nodes[1].layers == t.nodes[1].layers);
  CHECK(Topology::parse("{}", true).nodes.empty());
}

static void test_proto() {
  Message m;
  m.type = MsgType::Batch;
  m.batch = {{"model.layers.0", 7, 0}, {"model.layers.1", 7, 1}};
  std::vector<uint16_t> payload(12, 0x3c00);
  m.x.dtype = "f16";
  m.x.shape = {1, 3, 4};
  m.x.data = reinterpret_cast<const uint8_t*>(payload.data());
  m.x.nbytes = payload.size() * 2;
  const std::string body = encode_body(m);
  Message d = decode_body(reinterpret_cast<const uint8_t*>(body.data()), body.size());
  CHECK(d.type == MsgType::Batch && d.batch.size() == 2 && d.batch[1].block_idx == 1);
  CHECK(d.x.shape == m.x.shape && d.x.nbytes == m.x.nbytes);
  CHECK(std::memcmp(d.x.data, payload.data(), m.x.nbytes) == 0);
  uint8_t hdr[8];
  encode_header(1234, hdr);
  CHECK(decode_header(hdr) == 1234u);
  hdr[0] ^= 0xff;
  bool threw = false;
  try {
    decode_header(hdr);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
  // truncated body must throw, never read past the end
  threw = false;
  try {
    decode_body(reinterpret_cast<const uint8_t*>(body.data()), body.size() / 2);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_safetensors() {
  char tmpl[] = "/tmp/cake_selftest_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  const std::string path = std::string(dir) + "/model.safetensors";
  std::vector<float> a = {1.f, 2.f, 3.f, 4.f, 5.f, 6.f};
  std::vector<uint16_t> b = {1, 2, 3};
  write_safetensors(path, {{"a", "F32", {2, 3}, reinterpret_cast<const uint8_t*>(a.data()), 24},
                           {"b.weight", "BF16", {3}, reinterpret_cast<const uint8_t*>(b.data()), 6}},
                    {{"format", "pt"}});
  {
    SafeTensorsFile f(path);
    CHECK(f.has("a") && f.has("b.weight"));
    CHECK(f.tensor("a").shape == std::vector<uint64_t>({2, 3}));
    CHECK(std::memcmp(f.tensor("a").data, a.data(), 24) == 0);
    CHECK(f.metadata().at("format") == "pt");
    auto wm = load_weight_map(dir);
    CHECK(wm.size() == 2 && wm.at("b.weight") == "model.safetensors");
  }
  std::remove(path.c_str());
  rmdir(dir);
}

// echo-ish compute: returns the input tensor with every byte incremented
static OpResult compute(uint64_t, const std::vector<BatchItem>& ops, const RawTensor& x) {
  OpResult r;
  if (!ops.empty() && ops[0].layer_name == "bad") {
    r.error = "unknown layer bad";
    return r;
  }
  r.dtype = x.dtype;
  r.shape = x.shape;
  r.data.assign(reinterpret_cast<const char*>(x.data), x.nbytes);
  for (auto& c : r.data) c = (char)(c + 1);
  return r;
}

static Message roundtrip(int fd, const Message& m) {
  const std::string body = encode_body(m);
  send_frame(fd, reinterpret_cast<const uint8_t*>(body.data()), (uint32_t)body.size());
  static thread_local std::string keep;
  keep = recv_frame(fd);
  return decode_body(reinterpret_cast<const uint8_t*>(keep.data()), keep.size());
}

static void test_server() {
  WorkerInfo info;
  info.version = "selftest";
  info.device = "cpu";
  WorkerServer srv("127.0.0.1", 0, info, "selftest");
  std::atomic<int> resets{0}, drops{0};
  srv.set_compute(compute);
  srv.set_reset([&](uint64_t) { resets++; });
  srv.set_drop([&](uint64_t) { drops++; });
  srv.set_log([](const std::string&) {});
  srv.set_stats_every(3);
  std::thread accept_thr([&] { srv.serve(); });
  const int port = srv.port();

  constexpr int kClients = 6, kOps = 25;
  std::atomic<int> ok{0};
  std::vector<std::thread> cl;
  for (int c = 0; c < kClients; ++c)
    cl.emplace_back([&, c] {
      const int fd = tcp_connect("127.0.0.1", port, 5.0);
      Message hello;
      hello.type = MsgType::Hello;
      Message wi = roundtrip(fd, hello);
      if (wi.type != MsgType::WorkerInfo || wi.info.version != "selftest") return;
      std::vector<uint8_t> buf(64 + c);
      for (int i = 0; i < kOps; ++i) {
        for (size_t k = 0; k < buf.size(); ++k) buf[k] = (uint8_t)(k + i);
        Message op;
        op.type = MsgType::SingleOp;
        op.layer_name = "model.layers.0";
        op.x.dtype = "u8";
        op.x.shape = {buf.size()};
        op.x.data = buf.data();
        op.x.nbytes = buf.size();
        Message r = roundtrip(fd, op);
        bool good = r.type == MsgType::Tensor && r.x.nbytes == buf.size();
        for (size_t k = 0; good && k < buf.size(); ++k) good = r.x.data[k] == (uint8_t)(buf[k] + 1);
        if (!good) return;
      }
      Message bad;
      bad.type = MsgType::SingleOp;
      bad.layer_name = "bad";
      bad.x.dtype = "u8";
      bad.x.shape = {1};
      bad.x.data = buf.data();
      bad.x.nbytes = 1;
      if (roundtrip(fd, bad).type != MsgType::Error) return;
      Message ping;
      ping.type = MsgType::Ping;
      if (roundtrip(fd, ping).type != MsgType::Pong) return;
      Message reset;
      reset.type = MsgType::Reset;
      if (roundtrip(fd, reset).type != MsgType::Pong) return;
      tcp_close(fd);
      ok++;
    });
  for (auto& t : cl) t.join();
  CHECK(ok == kClients);
  CHECK(resets == kClients);

  // fault injection: the server drops the connection after 2 ops
  srv.set_drop_after(2);
  {
    const int fd = tcp_connect("127.0.0.1", port, 5.0);
    Message hello;
    hello.type = MsgType::Hello;
    roundtrip(fd, hello);
    uint8_t one = 1;
    Message op;
    op.type = MsgType::SingleOp;
    op.layer_name = "model.layers.0";
    op.x.dtype = "u8";
    op.x.shape = {1};
    op.x.data = &one;
    op.x.nbytes = 1;
    roundtrip(fd, op);
    roundtrip(fd, op);
    bool dropped = false;
    try {
      roundtrip(fd, op);
    } catch (const std::exception&) {
      dropped = true;
    }
    CHECK(dropped);
    tcp_close(fd);
  }
  srv.set_drop_after(0);

  // stop() with a connection still open and idle
  const int idle = tcp_connect("127.0.0.1", port, 5.0);
  Message hello;
  hello.type = MsgType::Hello;
  roundtrip(idle, hello);
  srv.stop();
  accept_thr.join();
  tcp_close(idle);
  CHECK(srv.stats().ops >= (uint64_t)kClients * kOps);
  CHECK(srv.stats().errors >= (uint64_t)kClients);
}

int main() {
  const struct {
    const char* name;
    void (*fn)();
  } tests[] = {{"topology", test_topology},
               {"proto", test_proto},
               {"safetensors", test_safetensors},
               {"server", test_server}};
  for (const auto& t : tests) {
    try {
      t.fn();
      std::printf("%-12s ok\n", t.name);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s threw: %s\n", t.name, e.what());
      ++g_fail;
    }
  }
  if (g_fail) std::fprintf(stderr, "%d failure(s)\n", g_fail);
  return g_fail ? 1 : 0;
}
