// cake-cli: the native entry point (master or worker), cake-cli/src/main.rs:8-63.
//
// Flags, defaults and choices follow cake-core/src/lib.rs:21-200 (SURVEY
// Appendix B) plus the MI355X extras; they are parsed and validated here
// (unknown flags, bad numbers, bad choices and a missing worker topology are
// rejected before any runtime starts; --help prints the table).  The topology
// is resolved with the native parser: a worker whose --name is not in the file
// serves the FIRST node (worker.rs:90-104), with a warning.  Then the process
// runs its role: the tensor compute (PyTorch-ROCm + the gfx950 HIP kernels) in
// an interpreter embedded in THIS process (embed.cpp), the worker's TCP
// control plane on the native WorkerServer.
#include <dlfcn.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../engine/llama_engine.h"
#include "embed.h"
#include "json.h"
#include "native_worker.h"
#include "server.h"
#include "topology.h"

using cake::PyArg;

namespace {

struct Flag {
  const char* name;     // --name
  const char* dest;     // argparse dest
  PyArg::Kind kind;
  const char* def;      // nullptr -> None
  const char* choices;  // "a|b|c" or nullptr
  bool is_switch;       // store_true
  const char* help;
};

const Flag kFlags[] = {
    {"--device", "device", PyArg::kInt, "0", nullptr, false, "GPU ordinal"},
    {"--mode", "mode", PyArg::kStr, "master", "master|worker", false, "role"},
    {"--name", "name", PyArg::kStr, nullptr, nullptr, false, "worker name (must be in the topology)"},
    {"--address", "address", PyArg::kStr, "127.0.0.1:10128", nullptr, false, "worker bind address"},
    {"--api", "api", PyArg::kStr, nullptr, nullptr, false,
     "serve the REST API on this address instead of one CLI generation"},
    {"--model", "model", PyArg::kStr, "./cake-data/Meta-Llama-3-8B/", nullptr, false, "model dir"},
    {"--topology", "topology", PyArg::kStr, "./cake-data/topology.yml", nullptr, false, "topology"},
    {"--prompt", "prompt", PyArg::kStr, "The sky is blue because ", nullptr, false, "prompt"},
    {"--system-prompt", "system_prompt", PyArg::kStr, "You are a helpful AI assistant.", nullptr,
     false, "system prompt"},
    {"--seed", "seed", PyArg::kInt, "299792458", nullptr, false, "sampling seed"},
    {"--sample-len", "sample_len", PyArg::kInt, "100", nullptr, false, "tokens to generate (-n)"},
    {"--temperature", "temperature", PyArg::kFloat, "1.0", nullptr, false, "<= 0: greedy"},
    {"--top-p", "top_p", PyArg::kFloat, nullptr, nullptr, false, "nucleus cutoff"},
    {"--top-k", "top_k", PyArg::kInt, nullptr, nullptr, false, "top-k cutoff"},
    {"--repeat-penalty", "repeat_penalty", PyArg::kFloat, "1.1", nullptr, false, "1 = off"},
    {"--repeat-last-n", "repeat_last_n", PyArg::kInt, "128", nullptr, false, "penalty window"},
    {"--dtype", "dtype", PyArg::kStr, nullptr, "f16|bf16|f32", false, "f16 (default), bf16, f32"},
    {"--cpu", "cpu", PyArg::kBool, "0", nullptr, true, "run on the CPU"},
    {"--model-type", "model_type", PyArg::kStr, "text-model", "text-model|image-model", false,
     "text or image model"},
    {"--sd-tokenizer", "sd_tokenizer", PyArg::kStr, nullptr, nullptr, false, ""},
    {"--sd-tokenizer-2", "sd_tokenizer_2", PyArg::kStr, nullptr, nullptr, false, ""},
    {"--sd-version", "sd_version", PyArg::kStr, "v1-5", "v1-5|v2-1|xl|turbo", false, ""},
    {"--sd-use-f16", "sd_use_f16", PyArg::kBool, "1", "true|false|1|0|yes|no|on|off", false, ""},
    {"--sd-width", "sd_width", PyArg::kInt, nullptr, nullptr, false, ""},
    {"--sd-height", "sd_height", PyArg::kInt, nullptr, nullptr, false, ""},
    {"--sd-sliced-attention-size", "sd_sliced_attention_size", PyArg::kInt, nullptr, nullptr, false,
     ""},
    {"--sd-clip", "sd_clip", PyArg::kStr, nullptr, nullptr, false, ""},
    {"--sd-clip2", "sd_clip2", PyArg::kStr, nullptr, nullptr, false, ""},
    {"--sd-vae", "sd_vae", PyArg::kStr, nullptr, nullptr, false, ""},
    {"--sd-unet", "sd_unet", PyArg::kStr, nullptr, nullptr, false, ""},
    {"--sd-use-flash-attention", "sd_use_flash_attention", PyArg::kBool, "0", nullptr, true, ""},
    {"--sd-image-prompt", "sd_image_prompt", PyArg::kStr,
     "A very realistic photo of a rusty robot walking on a sandy beach", nullptr, false, ""},
    {"--sd-uncond-prompt", "sd_uncond_prompt", PyArg::kStr, "", nullptr, false, ""},
    {"--sd-tracing", "sd_tracing", PyArg::kBool, "0", nullptr, true, ""},
    {"--sd-n-steps", "sd_n_steps", PyArg::kInt, nullptr, nullptr, false, ""},
    {"--sd-num-samples", "sd_num_samples", PyArg::kInt, "1", nullptr, false, ""},
    {"--sd-bsize", "sd_bsize", PyArg::kInt, "1", nullptr, false, ""},
    {"--sd-intermediary-images", "sd_intermediary_images", PyArg::kInt, "0", nullptr, false, ""},
    {"--sd-guidance-scale", "sd_guidance_scale", PyArg::kFloat, nullptr, nullptr, false, ""},
    {"--sd-img2img", "sd_img2img", PyArg::kStr, nullptr, nullptr, false, ""},
    {"--sd-img2img-strength", "sd_img2img_strength", PyArg::kFloat, "0.8", nullptr, false, ""},
    {"--sd-seed", "sd_seed", PyArg::kInt, nullptr, nullptr, false, ""},
    {"--transport", "transport", PyArg::kStr, "tcp", "tcp|rccl|loopback", false,
     "tcp, rccl (one rank per GPU) or loopback"},
    {"--parallel", "parallel", PyArg::kStr, "pp", "pp|tp", false,
     "rccl: pp = layer sharding (topology), tp = tensor parallel"},
    {"--hop", "hop", PyArg::kStr, "ipc", "ipc|dist", false,
     "rccl pp: device-side graph hops (ipc) or host-issued RCCL p2p (dist)"},
    {"--hop-dtype", "hop_dtype", PyArg::kStr, "f32", "f32|bf16", false, "ipc hop payload"},
    {"--max-seq-len", "max_seq_len", PyArg::kInt, "4096", nullptr, false, "KV cache length"},
    {"--no-graph", "no_graph", PyArg::kBool, "0", nullptr, true, "disable hipGraph decode"},
    {"--trace", "trace", PyArg::kStr, nullptr, nullptr, false, "chrome-trace JSON per generation"},
    {"--metrics", "metrics", PyArg::kStr, nullptr, nullptr, false, "append JSON stats lines"},
    {"--log-level", "log_level", PyArg::kStr, "info", "debug|info|warning|error", false, ""},
};

const Flag* find_flag(const std::string& n) {
  if (n == "-n") return find_flag("--sample-len");
  for (const auto& f : kFlags)
    if (n == f.name) return &f;
  return nullptr;
}

void usage() {
  std::printf("usage: cake-cli [flags]   (MI355X-native distributed inference)\n\n");
  for (const auto& f : kFlags) {
    std::printf("  %-28s %s", f.name, f.help);
    if (f.def && !f.is_switch) std::printf(" [default: %s]", f.def);
    if (f.choices) std::printf(" {%s}", f.choices);
    std::printf("\n");
  }
}

bool valid_number(const std::string& s, PyArg::Kind k) {
  if (s.empty()) return false;
  char* end = nullptr;
  if (k == PyArg::kInt) std::strtoll(s.c_str(), &end, 10);
  else std::strtod(s.c_str(), &end);
  return end && *end == '\0';
}

bool in_choices(const std::string& v, const char* choices) {
  std::string c = choices;
  size_t a = 0;
  while (a <= c.size()) {
    const size_t b = c.find('|', a);
    if (c.substr(a, b == std::string::npos ? std::string::npos : b - a) == v) return true;
    if (b == std::string::npos) break;
    a = b + 1;
  }
  return false;
}

// ---------------------------------------------------------------------------
// Native text generation: an all-local text model (no topology workers, no API server)
// runs on the native engine (libcake_engine.so, dlopen'ed: worker / image / API runs
// never load it) — checkpoint load, prefill, graph-replayed decode and token selection
// in C++; the embedded interpreter only tokenizes (cake_amd/native_bridge.py).
// CAKE_NATIVE=0 keeps the Python generator.  Output as Master.run: the streamed text,
// then the reference's rate line (master.rs:93-121) on stderr.
// ---------------------------------------------------------------------------
struct EngineApi {
  void* (*open)(const char*, const CakeEngineOpts*, char*, int32_t);
  void* (*open_pp)(const char*, const CakeEngineOpts*, const CakePipeOpts*, char*, int32_t);
  void* (*open_tp)(const char*, const CakeEngineOpts*, const CakeTPOpts*, char*, int32_t);
  void* (*open_remote)(const char*, const CakeEngineOpts*, const CakeRemoteOpts*, char*, int32_t);
  int32_t (*serve)(void*, char*, int32_t);
  int32_t (*generate)(void*, const int32_t*, int32_t, int32_t, const CakeEngineSampling*,
                      const int32_t*, int32_t, cake_engine_token_cb, void*, int32_t*, int32_t,
                      CakeEngineStats*, char*, int32_t);
  void (*close)(void*);
};

bool native_text_eligible(cake::PyArgs& o, bool text, bool worker, bool has_topology) {
  const char* env = std::getenv("CAKE_NATIVE");
  if (env && std::string(env) == "0") return false;
  const auto is = [&](const char* k, const char* v) { return o[k].value == v; };
  const bool common = text && o["api"].kind == PyArg::kNone && !is("cpu", "1") &&
                      !is("no_graph", "1") && o["trace"].kind == PyArg::kNone &&
                      o["metrics"].kind == PyArg::kNone &&
                      (o["dtype"].kind == PyArg::kNone || is("dtype", "f16") || is("dtype", "bf16"));
  if (is("transport", "rccl"))  // one process per GPU (torchrun env): layer-sharded pipeline
    return common && std::getenv("WORLD_SIZE") &&  // (pp, device hops) or tensor parallel
           ((is("parallel", "pp") && is("hop", "ipc")) || is("parallel", "tp"));
  (void)has_topology;  // topology workers: the engine's TCP client (native master)
  return common && !worker && is("transport", "tcp");
}

int env_int(const char* k, int def) {
  const char* v = std::getenv(k);
  return v ? std::atoi(v) : def;
}

struct StreamCtx {
  std::string model;
  std::vector<int32_t> eos;
};

int32_t stream_token(void* vctx, int32_t tok) {
  auto* c = static_cast<StreamCtx*>(vctx);
  for (int32_t e : c->eos)
    if (e == tok) return 0;  // EOS: nothing printed (the loop stops on it)
  cake::Json req = cake::Json::object();
  req.set("model", cake::Json::string(c->model));
  req.set("id", cake::Json::integer(tok));
  try {
    const std::string text = cake::call_python("cake_amd.native_bridge", "decode_token", req.dump());
    std::fwrite(text.data(), 1, text.size(), stdout);
    std::fflush(stdout);
  } catch (const std::exception&) {
  }
  return 0;
}

// Layer -> pipeline rank of the topology: node i (file order) runs on rank i + 1, every
// layer no node names stays on rank 0 (the master), as the reference's placement loop
// (llama.rs:205-220 with topology.rs:81-92).  Empty when no node places a layer.
std::vector<int32_t> owners_of(const cake::Topology* topo, int world, int num_layers) {
  std::vector<int32_t> own;
  if (!topo || topo->nodes.empty()) return own;
  if ((int)topo->nodes.size() > world - 1)
    throw std::runtime_error("topology has " + std::to_string(topo->nodes.size()) +
                             " workers but only " + std::to_string(world - 1) +
                             " worker ranks were launched");
  own.assign((size_t)num_layers, 0);
  bool any = false;
  const std::string pre = "model.layers.";
  for (size_t i = 0; i < topo->nodes.size(); ++i)
    for (const auto& l : topo->nodes[i].layers)
      if (l.rfind(pre, 0) == 0) {
        const int li = std::atoi(l.c_str() + pre.size());
        if (li >= 0 && li < num_layers) {
          own[(size_t)li] = (int32_t)(i + 1);
          any = true;
        }
      }
  if (!any) own.clear();
  return own;
}

int num_hidden_layers(const std::string& model_dir) {
  std::FILE* f = std::fopen((model_dir + "/config.json").c_str(), "rb");
  if (!f) throw std::runtime_error("cannot read " + model_dir + "/config.json");
  std::string txt;
  char buf[4096];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) txt.append(buf, n);
  std::fclose(f);
  return (int)cake::Json::parse(txt).get("num_hidden_layers").as_int();
}

int run_native_text(cake::PyArgs& o, const cake::Topology* topo) {
  const std::string lib = cake::package_root() + "/cake_amd/lib/libcake_engine.so";
  void* h = dlopen(lib.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "cake-cli: %s\n", dlerror());
    return 1;
  }
  EngineApi api{};
  api.open = reinterpret_cast<decltype(api.open)>(dlsym(h, "cake_engine_open"));
  api.generate = reinterpret_cast<decltype(api.generate)>(dlsym(h, "cake_engine_generate"));
  api.close = reinterpret_cast<decltype(api.close)>(dlsym(h, "cake_engine_close"));
  api.open_pp = reinterpret_cast<decltype(api.open_pp)>(dlsym(h, "cake_engine_open_pp"));
  api.serve = reinterpret_cast<decltype(api.serve)>(dlsym(h, "cake_engine_serve"));
  api.open_tp = reinterpret_cast<decltype(api.open_tp)>(dlsym(h, "cake_engine_open_tp"));
  api.open_remote = reinterpret_cast<decltype(api.open_remote)>(dlsym(h, "cake_engine_open_remote"));
  if (!api.open || !api.generate || !api.close || !api.open_pp || !api.serve || !api.open_tp ||
      !api.open_remote) {
    std::fprintf(stderr, "cake-cli: engine symbols missing in %s\n", lib.c_str());
    return 1;
  }
  // --transport rccl: this process is pipeline rank RANK of WORLD_SIZE (torchrun env);
  // the engine's control plane listens on MASTER_PORT + 1 (torchrun's store owns the port)
  const bool pipe = o["transport"].value == "rccl";
  const bool tp = pipe && o["parallel"].value == "tp";
  const int rank = pipe ? env_int("RANK", 0) : 0, world = pipe ? env_int("WORLD_SIZE", 1) : 1;
  const char* maddr = std::getenv("MASTER_ADDR");
  const std::string ctl = std::string(maddr ? maddr : "127.0.0.1") + ":" +
                          std::to_string(env_int("MASTER_PORT", 29500) + 1);
  StreamCtx ctx;
  ctx.model = o["model"].value;
  std::vector<int32_t> ids;
  // pp: the topology's placement (every rank parses the same file)
  std::vector<int32_t> owners;
  if (pipe && !tp && world > 1) {
    try {
      owners = owners_of(topo, world, num_hidden_layers(ctx.model));
    } catch (const std::exception& e) {
      std::fprintf(stderr, "cake-cli: rank %d: %s\n", rank, e.what());
      return 2;
    }
  }
  if (rank != 0) {  // worker rank: its layer shard, then serve rank 0
    const auto num = [&](const char* k, double def) {
      return o[k].kind == PyArg::kNone ? def : std::strtod(o[k].value.c_str(), nullptr);
    };
    CakeEngineOpts eo{(int32_t)num("max_seq_len", 4096), o["dtype"].value == "bf16" ? 0 : 1,
                      env_int("LOCAL_RANK", rank), 1};
    CakePipeOpts po{rank, world, ctl.c_str(), o["hop_dtype"].value == "bf16" ? 1 : 0, 60.0, 600.0,
                    owners.empty() ? nullptr : owners.data(), (int32_t)owners.size()};
    CakeTPOpts to{rank, world, ctl.c_str(), 60.0, 600.0};
    char err[1024] = {0};
    void* eng = tp ? api.open_tp(ctx.model.c_str(), &eo, &to, err, sizeof(err))
                   : api.open_pp(ctx.model.c_str(), &eo, &po, err, sizeof(err));
    if (!eng) {
      std::fprintf(stderr, "cake-cli: rank %d: %s\n", rank, err);
      return 1;
    }
    const int32_t rc = api.serve(eng, err, sizeof(err));
    if (rc) std::fprintf(stderr, "cake-cli: rank %d: %s\n", rank, err);
    api.close(eng);
    return rc ? 1 : 0;
  }
  try {
    cake::Json req = cake::Json::object();
    req.set("model", cake::Json::string(ctx.model));
    req.set("system", cake::Json::string(o["system_prompt"].value));
    req.set("prompt", cake::Json::string(o["prompt"].value));
    const cake::Json r = cake::Json::parse(
        cake::call_python("cake_amd.native_bridge", "encode_chat", req.dump()));
    for (const auto& x : r.get("ids").items()) ids.push_back((int32_t)x.as_int());
    for (const auto& x : r.get("eos").items()) ctx.eos.push_back((int32_t)x.as_int());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "cake-cli: tokenizer: %s\n", e.what());
    return 1;
  }
  const auto num = [&](const char* k, double def) {
    return o[k].kind == PyArg::kNone ? def : std::strtod(o[k].value.c_str(), nullptr);
  };
  CakeEngineOpts eo{};
  eo.max_seq = (int32_t)num("max_seq_len", 4096);
  eo.dtype = o["dtype"].value == "bf16" ? 0 : 1;  // reference default: f16
  eo.device = pipe ? env_int("LOCAL_RANK", 0) : (int32_t)num("device", 0);
  eo.steps_per_graph = 1;
  char err[1024] = {0};
  const auto t0 = std::chrono::steady_clock::now();
  CakePipeOpts po{0, world, ctl.c_str(), o["hop_dtype"].value == "bf16" ? 1 : 0, 60.0, 600.0,
                  owners.empty() ? nullptr : owners.data(), (int32_t)owners.size()};
  CakeTPOpts to{0, world, ctl.c_str(), 60.0, 600.0};
  // --transport tcp with topology workers: the master's TCP client (llama.rs:205-220:
  // each layer a node names runs on that node; contiguous runs go as one Batch)
  std::vector<int32_t> worker_of;
  std::vector<const char*> hosts;
  if (!pipe && topo && !topo->nodes.empty()) {
    int L = 0;
    try {
      L = num_hidden_layers(ctx.model);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "cake-cli: %s\n", e.what());
      return 1;
    }
    worker_of.assign((size_t)L, -1);
    for (int l = 0; l < L; ++l) {
      const cake::TopoNode* nd = topo->node_for_layer("model.layers." + std::to_string(l));
      if (nd) worker_of[(size_t)l] = (int32_t)(nd - topo->nodes.data());
    }
    for (const auto& nd : topo->nodes) hosts.push_back(nd.host.c_str());
  }
  CakeRemoteOpts ro{worker_of.data(), (int32_t)worker_of.size(), hosts.data(),
                    (int32_t)hosts.size(), 120.0};
  void* eng = world > 1 ? (tp ? api.open_tp(ctx.model.c_str(), &eo, &to, err, sizeof(err))
                              : api.open_pp(ctx.model.c_str(), &eo, &po, err, sizeof(err)))
              : !worker_of.empty() ? api.open_remote(ctx.model.c_str(), &eo, &ro, err, sizeof(err))
                                   : api.open(ctx.model.c_str(), &eo, err, sizeof(err));
  if (!eng) {
    std::fprintf(stderr, "cake-cli: native engine: %s\n", err);
    return 1;
  }
  const double load_s =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::fprintf(stderr, "[cake-cli] native engine: model loaded in %.1f s (%zu prompt tokens)%s\n",
               load_s, ids.size(),
               worker_of.empty() ? "" : ", native master over TCP workers");
  CakeEngineSampling smp{};
  smp.temperature = (float)num("temperature", 1.0);
  smp.top_k = (int32_t)num("top_k", 0);
  smp.top_p = (float)num("top_p", 0.0);
  smp.seed = (uint64_t)std::strtoull(o["seed"].value.c_str(), nullptr, 10);
  smp.repeat_penalty = (float)num("repeat_penalty", 1.1);
  smp.repeat_last_n = (int32_t)num("repeat_last_n", 128);
  const int32_t n = (int32_t)num("sample_len", 100);
  const int32_t room = eo.max_seq - (int32_t)ids.size() - 3;
  const int32_t max_new = n < room ? n : room;
  std::vector<int32_t> out((size_t)(max_new > 0 ? max_new : 1));
  CakeEngineStats st{};
  const int32_t rc = api.generate(eng, ids.data(), (int32_t)ids.size(), max_new, &smp,
                                  ctx.eos.data(), (int32_t)ctx.eos.size(), stream_token, &ctx,
                                  out.data(), (int32_t)out.size(), &st, err, sizeof(err));
  std::fputc('\n', stdout);
  std::fflush(stdout);
  if (rc != 0) {
    std::fprintf(stderr, "cake-cli: native engine: %s\n", err);
    api.close(eng);
    return 1;
  }
  std::fprintf(stderr, "[cake-cli] %d tokens generated (%.2f token/s) p50=%.2fms p99=%.2fms "
               "ttft=%.1fms\n", st.n_generated, st.tokens_per_s, st.p50_ms, st.p99_ms,
               st.prefill_s * 1e3);
  api.close(eng);
  return 0;
}

// ---------------------------------------------------------------------------
// Native TCP worker (--mode worker, text model): runtime/native_worker.cpp.
// ---------------------------------------------------------------------------
bool native_worker_eligible(cake::PyArgs& o, bool text, bool worker) {
  const char* env = std::getenv("CAKE_NATIVE");
  if (env && std::string(env) == "0") return false;
  return text && worker && o["cpu"].value != "1" && o["transport"].value == "tcp" &&
         (o["dtype"].kind == PyArg::kNone || o["dtype"].value == "f16" ||
          o["dtype"].value == "bf16");
}

// image model: the native SD worker serves unet / clip / clip2 / vae (decode) components
bool native_sd_worker_eligible(cake::PyArgs& o, bool text, bool worker,
                               const cake::TopoNode& node) {
  const char* env = std::getenv("CAKE_NATIVE");
  if (env && std::string(env) == "0") return false;
  return !text && worker && o["cpu"].value != "1" && o["transport"].value == "tcp" &&
         (o["dtype"].kind == PyArg::kNone || o["dtype"].value == "f16" ||
          o["dtype"].value == "bf16") &&
         cake::native_sd_components(node) && cake::native_engine_available();
}

int run_native_sd_worker(cake::PyArgs& o, const cake::TopoNode& node) {
  cake::NativeWorkerOpts w;
  w.model_dir = o["model"].value;
  w.address = o["address"].value;
  w.device = o["device"].kind == PyArg::kNone ? 0 : std::atoi(o["device"].value.c_str());
  w.bf16 = o["dtype"].value == "bf16";
  w.sd_version = o["sd_version"].value;
  if (o["sd_width"].kind != PyArg::kNone) w.sd_width = std::atoi(o["sd_width"].value.c_str());
  if (o["sd_height"].kind != PyArg::kNone) w.sd_height = std::atoi(o["sd_height"].value.c_str());
  const char* keys[4] = {"sd_unet", "sd_vae", "sd_clip", "sd_clip2"};
  for (int k = 0; k < 4; ++k)
    if (o[keys[k]].kind != PyArg::kNone) w.sd_paths[k] = o[keys[k]].value;
  return cake::run_native_sd_worker(w, node);
}

int run_native_worker(cake::PyArgs& o, const cake::TopoNode& node) {
  cake::NativeWorkerOpts w;
  w.model_dir = o["model"].value;
  w.address = o["address"].value;
  w.device = o["device"].kind == PyArg::kNone ? 0 : std::atoi(o["device"].value.c_str());
  w.max_seq = o["max_seq_len"].kind == PyArg::kNone ? 4096 : std::atoi(o["max_seq_len"].value.c_str());
  w.bf16 = o["dtype"].value == "bf16";
  return cake::run_native_worker(w, node);
}

}  // namespace

int main(int argc, char** argv) {
  cake::PyArgs opts;
  for (const auto& f : kFlags) {
    PyArg a;
    if (f.def == nullptr) a.kind = PyArg::kNone;
    else { a.kind = f.kind; a.value = f.def; }
    opts[f.dest] = a;
  }
  if (const char* lv = std::getenv("CAKE_LOG")) opts["log_level"] = PyArg{PyArg::kStr, lv};
  for (int i = 1; i < argc; ++i) {
    std::string arg = argv[i];
    if (arg == "-h" || arg == "--help") { usage(); return 0; }
    std::string val;
    bool has_val = false;
    const auto eq = arg.find('=');
    if (arg.rfind("--", 0) == 0 && eq != std::string::npos) {
      val = arg.substr(eq + 1);
      arg = arg.substr(0, eq);
      has_val = true;
    }
    const Flag* f = find_flag(arg);
    if (!f) { std::fprintf(stderr, "cake-cli: unknown flag %s (see --help)\n", arg.c_str()); return 2; }
    if (f->is_switch) {
      if (has_val) { std::fprintf(stderr, "cake-cli: %s takes no value\n", f->name); return 2; }
      opts[f->dest] = PyArg{PyArg::kBool, "1"};
      continue;
    }
    if (!has_val) {
      if (i + 1 >= argc) { std::fprintf(stderr, "cake-cli: %s needs a value\n", f->name); return 2; }
      val = argv[++i];
    }
    if ((f->kind == PyArg::kInt || f->kind == PyArg::kFloat) && !valid_number(val, f->kind)) {
      std::fprintf(stderr, "cake-cli: %s: invalid number '%s'\n", f->name, val.c_str());
      return 2;
    }
    if (f->choices && !in_choices(val, f->choices)) {
      std::fprintf(stderr, "cake-cli: %s: '%s' not in {%s}\n", f->name, val.c_str(), f->choices);
      return 2;
    }
    if (f->kind == PyArg::kBool) {  // --sd-use-f16 true|false
      opts[f->dest] = PyArg{PyArg::kBool, (val == "true" || val == "1" || val == "yes" ||
                                           val == "on") ? "1" : "0"};
      continue;
    }
    opts[f->dest] = PyArg{f->kind, val};
  }
  // ---- topology (native parser): validate placement before any runtime starts
  const bool text = opts["model_type"].value == "text-model";
  const std::string topo_path = opts["topology"].value;
  const bool worker = opts["mode"].value == "worker";
  bool has_topology = false;
  cake::TopoNode worker_node;
  std::unique_ptr<cake::Topology> topology;
  if (access(topo_path.c_str(), R_OK) == 0) {
    try {
      const cake::Topology topo = cake::Topology::from_path(topo_path, text);
      size_t layers = 0;
      for (const auto& n : topo.nodes) layers += n.layers.size();
      std::fprintf(stderr, "[cake-cli] topology %s: %zu node(s), %zu placed unit(s)\n",
                   topo_path.c_str(), topo.nodes.size(), layers);
      has_topology = !topo.nodes.empty();
      topology.reset(new cake::Topology(topo));
      if (worker) {
        if (topo.nodes.empty()) { std::fprintf(stderr, "cake-cli: topology has no workers\n"); return 2; }
        const PyArg& nm = opts["name"];
        if (nm.kind == PyArg::kNone || !topo.find(nm.value))
          std::fprintf(stderr, "[cake-cli] worker name %s not in the topology: serving the FIRST "
                       "node '%s'\n", nm.kind == PyArg::kNone ? "(none)" : nm.value.c_str(),
                       topo.nodes[0].name.c_str());
        const cake::TopoNode* nd = nm.kind == PyArg::kNone ? nullptr : topo.find(nm.value);
        worker_node = nd ? *nd : topo.nodes[0];
      }
    } catch (const std::exception& e) {
      std::fprintf(stderr, "cake-cli: bad topology %s: %s\n", topo_path.c_str(), e.what());
      return 2;
    }
  } else if (worker) {
    std::fprintf(stderr, "cake-cli: worker mode needs a topology (%s not found)\n",
                 topo_path.c_str());
    return 2;
  }
  if (native_text_eligible(opts, text, worker, has_topology))
    return run_native_text(opts, topology.get());
  if (native_worker_eligible(opts, text, worker)) return run_native_worker(opts, worker_node);
  if (native_sd_worker_eligible(opts, text, worker, worker_node))
    return run_native_sd_worker(opts, worker_node);
  return cake::run_embedded(opts);
}
