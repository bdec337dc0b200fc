// Host self-test of the native workers' control plane (native_worker.cpp over
// server.cpp / net.cpp / proto.cpp) against the stub engine (stub_engine.cpp, loaded
// through CAKE_ENGINE_LIB): no GPU, so it runs plain, under ASan+UBSan and under TSan
// (scripts/sanitize_runtime.sh, tests/test_sanitizers_cpu.py).
//
// Text worker: three masters at once, each a prefill Batch and decode Batches on its
// own KV session (values checked against the stub's closed form), rows of the wrong
// width / a position past 2^31 / a layer the node does not own / a non-float tensor
// (each an Error reply, the connection still usable), a master that disconnects with a
// request in flight, one that closes mid-frame, Ping and Reset; then stop() with the
// engine closed after every connection thread has been joined.  The engine counts
// overlapping calls: the worker's compute lock must leave none.
// SD worker: clip / unet / vae requests from two masters, and malformed packs (a NaN or
// negative header, a size past the buffer, an empty timestep item, a 1-channel latent).
#include <dlfcn.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/native_worker.h"
#include "../runtime/net.h"
#include "../runtime/proto.h"
#include "../runtime/server.h"

using namespace cake;

static std::atomic<int> g_fail{0};
#define CHECK(c)                                                                   \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);     \
      ++g_fail;                                                                    \
    }                                                                              \
  } while (0)

constexpr int kH = 64;  // the stub's hidden size

static Message roundtrip(int fd, const Message& m) {
  const std::string body = encode_body(m);
  send_frame(fd, reinterpret_cast<const uint8_t*>(body.data()), (uint32_t)body.size());
  static thread_local std::string keep;
  keep = recv_frame(fd);
  return decode_body(reinterpret_cast<const uint8_t*>(keep.data()), keep.size());
}

static int hello(int port) {
  const int fd = tcp_connect("127.0.0.1", port, 5.0);
  Message h;
  h.type = MsgType::Hello;
  const Message wi = roundtrip(fd, h);
  CHECK(wi.type == MsgType::WorkerInfo);
  return fd;
}

static Message batch(const std::vector<int>& layers, uint64_t pos, const std::vector<float>& x,
                     std::vector<uint64_t> shape) {
  Message m;
  m.type = MsgType::Batch;
  for (int l : layers) m.batch.push_back({"model.layers." + std::to_string(l), pos, 0});
  m.x.dtype = "f32";
  m.x.shape = std::move(shape);
  m.x.data = reinterpret_cast<const uint8_t*>(x.data());
  m.x.nbytes = x.size() * 4;
  return m;
}

static float expect_add(const std::vector<int>& layers, int pos) {
  float a = 0.f;
  for (int l : layers) a += (l + 1) * 0.5f + pos * 0.25f;
  return a;
}

// runs `serve` on a thread, returns once the server listens
struct Running {
  std::atomic<WorkerServer*> srv{nullptr};
  std::atomic<int> rc{-1};
  std::thread thr;
  template <class F>
  explicit Running(F serve) {
    thr = std::thread([this, serve] { rc = serve([this](WorkerServer& s) { srv = &s; }); });
    for (int i = 0; i < 500 && !srv.load() && rc.load() < 0; ++i) usleep(10000);
    if (!srv.load()) throw std::runtime_error("worker did not start");
  }
  int port() const { return srv.load()->port(); }
  int stop() {
    srv.load()->stop();
    thr.join();
    return rc.load();
  }
};

static void test_text_worker() {
  TopoNode node;
  node.name = "w1";
  for (int l = 0; l < 4; ++l) node.layers.push_back("model.layers." + std::to_string(l));
  Running run([&](std::function<void(WorkerServer&)> ready) {
    NativeWorkerOpts o;
    o.model_dir = "stub";
    o.address = "127.0.0.1:0";
    o.log_tag = "worker_selftest";
    o.on_serving = ready;
    return run_native_worker(o, node);
  });
  const int port = run.port();

  constexpr int kMasters = 3, kDecode = 12, kT = 5;
  std::atomic<int> ok{0};
  std::vector<std::thread> ms;
  for (int c = 0; c < kMasters; ++c)
    ms.emplace_back([&, c] {
      const int fd = hello(port);
      bool good = true;
      // prefill: T rows through all four layers at position 0
      std::vector<float> x((size_t)kT * kH);
      for (size_t i = 0; i < x.size(); ++i) x[i] = 0.01f * (float)i + c;
      Message r = roundtrip(fd, batch({0, 1, 2, 3}, 0, x, {1, (uint64_t)kT, (uint64_t)kH}));
      good &= r.type == MsgType::Tensor && r.x.nbytes == x.size() * 4;
      if (good) {
        const float* y = reinterpret_cast<const float*>(r.x.data);
        for (int t = 0; t < kT && good; ++t)
          for (int k = 0; k < kH; ++k) {
            float want = x[(size_t)t * kH + k];
            for (int l = 0; l < 4; ++l) want += (l + 1) * 0.5f + t * 0.25f;
            good &= std::fabs(y[(size_t)t * kH + k] - want) < 1e-3f;
          }
      }
      // decode: one row per step, two runs of the node's layers (two Batch items each)
      for (int s = 0; s < kDecode && good; ++s) {
        const int pos = kT + s;
        std::vector<float> row(kH, 1.f + c);
        r = roundtrip(fd, batch({0, 1, 2, 3}, (uint64_t)pos, row, {1, 1, (uint64_t)kH}));
        good &= r.type == MsgType::Tensor && r.x.nbytes == kH * 4;
        if (good) {
          const float* y = reinterpret_cast<const float*>(r.x.data);
          good &= std::fabs(y[7] - (row[7] + expect_add({0, 1, 2, 3}, pos))) < 1e-3f;
        }
      }
      // malformed requests: an Error reply each, and the session stays usable
      std::vector<float> narrow(kH - 1, 0.f), wide((size_t)kH * 3 + 5, 0.f);
      good &= roundtrip(fd, batch({0}, kT + kDecode, narrow, {1, 1, (uint64_t)kH - 1})).type ==
              MsgType::Error;
      good &= roundtrip(fd, batch({0}, kT + kDecode, wide, {1, (uint64_t)wide.size()})).type ==
              MsgType::Error;
      std::vector<float> row(kH, 0.f);
      good &= roundtrip(fd, batch({0}, 1ull << 40, row, {1, 1, (uint64_t)kH})).type ==
              MsgType::Error;
      good &= roundtrip(fd, batch({7}, kT + kDecode, row, {1, 1, (uint64_t)kH})).type ==
              MsgType::Error;
      {
        Message m = batch({0}, kT + kDecode, row, {1, 1, (uint64_t)kH});
        m.x.dtype = "u8";
        m.x.nbytes = kH;  // consistent bytes, wrong dtype
        good &= roundtrip(fd, m).type == MsgType::Error;
      }
      r = roundtrip(fd, batch({2, 3}, kT + kDecode, row, {1, 1, (uint64_t)kH}));
      good &= r.type == MsgType::Tensor;
      Message ping;
      ping.type = MsgType::Ping;
      good &= roundtrip(fd, ping).type == MsgType::Pong;
      Message reset;
      reset.type = MsgType::Reset;
      good &= roundtrip(fd, reset).type == MsgType::Pong;
      tcp_close(fd);
      if (good) ok++;
    });
  // a master that disconnects with a request in flight, and one that closes mid-frame
  std::thread gone([&] {
    const int fd = hello(port);
    std::vector<float> x((size_t)kT * kH, 0.5f);
    const Message m = batch({0, 1}, 0, x, {1, (uint64_t)kT, (uint64_t)kH});
    const std::string body = encode_body(m);
    send_frame(fd, reinterpret_cast<const uint8_t*>(body.data()), (uint32_t)body.size());
    tcp_close(fd);
    const int fd2 = hello(port);  // the frame's header and half its body, then close
    const std::string b2 = encode_body(batch({0}, 0, x, {1, (uint64_t)kT, (uint64_t)kH}));
    uint8_t hdr[8];
    encode_header((uint32_t)b2.size(), hdr);
    CHECK(::write(fd2, hdr, 8) == 8);
    CHECK(::write(fd2, b2.data(), b2.size() / 2) == (ssize_t)(b2.size() / 2));
    (void)::shutdown(fd2, SHUT_WR);
    tcp_close(fd2);
  });
  for (auto& t : ms) t.join();
  gone.join();
  CHECK(ok == kMasters);
  // one more master after the others are gone: the worker still serves
  {
    const int fd = hello(port);
    std::vector<float> row(kH, 2.f);
    const Message r = roundtrip(fd, batch({1}, 0, row, {1, 1, (uint64_t)kH}));
    CHECK(r.type == MsgType::Tensor);
    tcp_close(fd);
  }
  const int idle = hello(port);  // stop() with an idle connection open
  CHECK(run.stop() == 0);
  tcp_close(idle);
}

// ---- SD worker --------------------------------------------------------------------------
static std::vector<float> pack(const std::vector<std::pair<std::vector<uint64_t>, std::vector<float>>>& items) {
  std::vector<float> f{(float)items.size()};
  for (const auto& it : items) {
    f.push_back((float)it.first.size());
    for (auto d : it.first) f.push_back((float)d);
    f.insert(f.end(), it.second.begin(), it.second.end());
  }
  return f;
}

static Message single(const std::string& name, const std::vector<float>& f) {
  Message m;
  m.type = MsgType::SingleOp;
  m.layer_name = name;
  m.x.dtype = "f32";
  m.x.shape = {(uint64_t)f.size()};
  m.x.data = reinterpret_cast<const uint8_t*>(f.data());
  m.x.nbytes = f.size() * 4;
  return m;
}

static void test_sd_worker() {
  TopoNode node;
  node.name = "sd";
  node.layers = {"unet", "vae", "clip"};
  Running run([&](std::function<void(WorkerServer&)> ready) {
    NativeWorkerOpts o;
    o.model_dir = "stub";
    o.address = "127.0.0.1:0";
    o.log_tag = "worker_selftest";
    o.on_serving = ready;
    return run_native_sd_worker(o, node);
  });
  const int port = run.port();
  constexpr int W = 64, H = 64, Dc = 16, nl = 4 * (H / 8) * (W / 8);
  std::atomic<int> ok{0};
  std::vector<std::thread> ms;
  for (int c = 0; c < 2; ++c)
    ms.emplace_back([&, c] {
      const int fd = hello(port);
      bool good = true;
      std::vector<float> ids(77, 3.f + c);
      Message r = roundtrip(fd, single("clip", ids));
      good &= r.type == MsgType::Tensor && r.x.nbytes == 77 * 8 * 4;
      std::vector<float> lat(nl, 1.f), ctx(77 * Dc, 0.f), ts{10.f};
      const auto unet = pack({{{1, 4, H / 8, W / 8}, lat}, {{1, 77, Dc}, ctx}, {{1}, ts}});
      r = roundtrip(fd, single("unet", unet));
      good &= r.type == MsgType::Tensor && r.x.nbytes == nl * 4;
      if (good) good &= std::fabs(reinterpret_cast<const float*>(r.x.data)[5] - 10.5f) < 1e-4f;
      const auto dec = pack({{{1}, {0.f}}, {{1, 4, H / 8, W / 8}, lat}});
      r = roundtrip(fd, single("vae", dec));
      good &= r.type == MsgType::Tensor && r.x.nbytes == 3u * H * W * 4;
      std::vector<float> img(3 * H * W, 0.25f);
      const auto enc = pack({{{1}, {1.f}}, {{1, 3, H, W}, img}});
      r = roundtrip(fd, single("vae", enc));
      good &= r.type == MsgType::Tensor && r.x.nbytes == nl * 4;
      // malformed packs
      std::vector<float> bad = unet;
      bad[0] = std::numeric_limits<float>::quiet_NaN();
      good &= roundtrip(fd, single("unet", bad)).type == MsgType::Error;
      bad = unet;
      bad[1] = -4.f;
      good &= roundtrip(fd, single("unet", bad)).type == MsgType::Error;
      bad = unet;
      bad[2] = 1e9f;  // a dimension far past the buffer
      good &= roundtrip(fd, single("unet", bad)).type == MsgType::Error;
      const auto no_t = pack({{{1, 4, H / 8, W / 8}, lat}, {{1, 77, Dc}, ctx}, {{0}, {}}});
      good &= roundtrip(fd, single("unet", no_t)).type == MsgType::Error;
      const auto one_ch = pack({{{1}, {0.f}}, {{1, 1, H / 8, W / 8}, std::vector<float>(nl / 4)}});
      good &= roundtrip(fd, single("vae", one_ch)).type == MsgType::Error;
      const auto no_dir = pack({{{0}, {}}, {{1, 4, H / 8, W / 8}, lat}});
      good &= roundtrip(fd, single("vae", no_dir)).type == MsgType::Error;
      good &= roundtrip(fd, single("clip", std::vector<float>(76, 1.f))).type == MsgType::Error;
      tcp_close(fd);
      if (good) ok++;
    });
  for (auto& t : ms) t.join();
  CHECK(ok == 2);
  CHECK(run.stop() == 0);
}

int main() {
  const char* lib = std::getenv("CAKE_ENGINE_LIB");
  if (!lib || !*lib) {
    std::fprintf(stderr, "CAKE_ENGINE_LIB must name the stub engine\n");
    return 2;
  }
  const struct {
    const char* name;
    void (*fn)();
  } tests[] = {{"text_worker", test_text_worker}, {"sd_worker", test_sd_worker}};
  for (const auto& t : tests) {
    try {
      t.fn();
      std::printf("%-12s ok\n", t.name);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s threw: %s\n", t.name, e.what());
      ++g_fail;
    }
  }
  void* h = dlopen(lib, RTLD_NOW | RTLD_NOLOAD);
  auto overlaps = h ? reinterpret_cast<int (*)()>(dlsym(h, "stub_engine_overlaps")) : nullptr;
  CHECK(overlaps != nullptr);
  if (overlaps) CHECK(overlaps() == 0);
  if (h) dlclose(h);
  if (g_fail) std::fprintf(stderr, "%d failure(s)\n", g_fail.load());
  return g_fail ? 1 : 0;
}
