// Native decode driver interface (graph_loop.cpp): the replay / read-back / EOS loop
// shared by the Python front (ops/graph_loop.py, ctypes mirror of these structs) and
// the native engine (csrc/engine/llama_engine.cpp).
#pragma once
#include <stdint.h>

extern "C" {
typedef int32_t (*cake_token_cb)(void* ctx, int32_t token);
typedef int32_t (*cake_announce_cb)(void* ctx, int32_t first, int32_t count);

struct CakeLoopSpec {
  void* const* execs;         // hipGraphExec_t per position bucket
  int32_t n_execs;
  const int32_t* bucket_of;   // [n_len]: bucket for the live length after a replay
  int32_t n_len;
  int32_t k;                  // decode steps per replay (tokens per graph)
  const int32_t* hist;        // device token history, or null (worker: no read-back)
  int32_t base;               // history index of the first token this run generates
  int32_t pos;                // host mirror of the device position (last written row)
  int32_t n;                  // tokens to generate (replays = ceil(n / k))
  int32_t chunk;              // replays per announce (0: everything at once)
  const int32_t* eos;         // EOS ids (host)
  int32_t n_eos;
  cake_token_cb on_token;     // optional; non-zero return = stop
  void* token_ctx;
  cake_announce_cb announce;  // optional; non-zero return = error
  void* announce_ctx;
  void* stream;               // hipStream_t
  int32_t* out_tokens;        // host [out_cap]
  float* out_ms;              // host [out_cap]: device time per token (ms)
  int32_t out_cap;
};

struct CakeLoopResult {
  int32_t n_tokens;   // tokens reported (stopped at EOS inclusive)
  int32_t replays;    // graph replays enqueued
  int32_t pos;        // host position after the last enqueued replay
  int32_t stopped;    // 1 = EOS / callback stop, 0 = ran to n
  double wall_s;
};
}

extern "C" int cake_graph_decode(const CakeLoopSpec* s, CakeLoopResult* r);
