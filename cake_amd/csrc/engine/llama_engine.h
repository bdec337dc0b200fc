// Native Llama text-generation engine: C ABI (libcake_engine.so).
//
// The whole text path of one all-local model without Python: checkpoint (safetensors,
// HF names) -> device weights, MFMA-GEMM prefill, hipGraph-captured decode steps
// (hipStreamBeginCapture over the gfx950 kernels' C entry points), device token
// selection, and the per-token replay loop (graph_loop.cpp).  Reference: the master's
// generation loop cake-core/src/cake/master.rs:80-124 and the Llama generator
// cake-core/src/models/llama3/llama.rs:72-138, 277-341.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t (*cake_engine_token_cb)(void* ctx, int32_t token);  // non-zero = stop

struct CakeEngineOpts {
  int32_t max_seq;          // KV-cache length (prompt + generated tokens)
  int32_t dtype;            // 0 = bf16, 1 = f16
  int32_t device;           // GPU ordinal
  int32_t steps_per_graph;  // decode steps per graph replay (greedy only; >= 1)
  int32_t init;             // 0: the checkpoint's safetensors; 1: seeded random-normal
                            // weights of the config.json architecture (benchmarks)
  int32_t reserved;
  uint64_t seed;            // init = 1: weight seed
};

// Layer-sharded pipeline over one process per GPU.  Placement: `owners[l]` is the rank
// running layer l (a topology: node i -> rank i + 1, unplaced layers on rank 0), any
// pattern — every maximal run of consecutive layers on one rank is one stop of the
// token's walk (llama.rs:95-114); no owner map = contiguous shards, rank 0 lighter by
// the head.  Rank 0 always holds the embedding and the head.  Each decode step's
// hidden state moves between stops by device-side hops (hop.hip, one IPC-mapped inbox
// per edge of the walk: no host in the step), prefill rows through IPC-mapped buffers;
// the control plane (IPC handles, prefill relay, replay announcements) is TCP to rank 0
// at master_addr.  Every edge is self-tested with a tagged pattern at start-up.
struct CakePipeOpts {
  int32_t rank, world;
  const char* master_addr;   // "host:port" rank 0 listens on
  int32_t hop_bf16;          // 1: bf16 hop payload (half the bytes)
  double hop_timeout_s;      // a hop receive that waits longer sets the error word
  double connect_timeout_s;  // workers: how long to retry reaching rank 0
  const int32_t* owners;     // [n_owners == num_hidden_layers] or null
  int32_t n_owners;
};

// Tensor parallel over one process per GPU: every rank holds 1/world of every layer (its
// query / KV heads, its slice of the intermediate rows) and of the vocabulary; the
// decode step's two all-reduces per layer and the token selection are device-side
// (allreduce.hip, IPC-mapped inboxes) inside each rank's captured graph; prefill sums go
// through IPC-mapped slabs.  Rank 0 generates; the others serve (cake_engine_serve).
struct CakeTPOpts {
  int32_t rank, world;       // world <= 8
  const char* master_addr;   // "host:port" rank 0 listens on
  double timeout_s;          // all-reduce wait bound (error word instead of a hang)
  double connect_timeout_s;
};

// Master over TCP workers (the reference's Client, cake-core/src/cake/client.rs:23-133):
// layer l runs on worker worker_of[l] ("host:port", a topology node's host) or locally
// (-1).  One connection per worker (Hello -> WorkerInfo at open); every contiguous run of
// one worker's layers is one Batch round trip per token (llama.rs:95-114), the hidden
// rows travel as f32 tensors.  The decode step runs eagerly (a host round trip sits
// inside it); local runs, the head and the token choice are the same kernels.
struct CakeRemoteOpts {
  const int32_t* worker_of;     // [n_layers == num_hidden_layers]
  int32_t n_layers;
  const char* const* workers;   // [n_workers] "host:port"
  int32_t n_workers;
  double timeout_s;             // connect / reply wait bound
};

struct CakeEngineSampling {
  float temperature;        // <= 0: greedy
  int32_t top_k;            // 0: off
  float top_p;              // 0 or >= 1: off
  uint64_t seed;
  float repeat_penalty;     // 1: off
  int32_t repeat_last_n;
};

struct CakeEngineStats {
  int32_t n_prompt;
  int32_t n_generated;
  double prefill_s;         // embed + layers + head + first token (host wall)
  double decode_s;          // generated tokens after the first (host wall)
  double tokens_per_s;      // (n_generated - 1) / decode_s: the reference's rate
  float p50_ms, p99_ms;     // device time per decode token
};

// config.json + safetensors of `model_dir`; null on failure (message in err).
void* cake_engine_open(const char* model_dir, const struct CakeEngineOpts* opts, char* err,
                       int32_t errlen);
// Pipeline rank (see CakePipeOpts): loads only its layer shard, joins the ring.
void* cake_engine_open_pp(const char* model_dir, const struct CakeEngineOpts* opts,
                          const struct CakePipeOpts* pipe, char* err, int32_t errlen);
// Tensor-parallel rank (see CakeTPOpts).
void* cake_engine_open_tp(const char* model_dir, const struct CakeEngineOpts* opts,
                          const struct CakeTPOpts* tp, char* err, int32_t errlen);
// Master with TCP workers (see CakeRemoteOpts): embedding, head and the local layers here.
void* cake_engine_open_remote(const char* model_dir, const struct CakeEngineOpts* opts,
                              const struct CakeRemoteOpts* remote, char* err, int32_t errlen);
// Workers (rank > 0): serve rank 0's control messages until it closes; 0 or an error.
int32_t cake_engine_serve(void* engine, char* err, int32_t errlen);
// TCP worker (topology node): only `layers` (global indices), no embedding / head.
void* cake_engine_open_layers(const char* model_dir, const struct CakeEngineOpts* opts,
                              const int32_t* layers, int32_t n_layers, char* err,
                              int32_t errlen);
// Run `layers` over hidden [T, H] f32 (host memory, in place) at positions pos0.. with
// the KV cache of `session` (created on first use); 0 or an error.
int32_t cake_engine_forward(void* engine, uint64_t session, const int32_t* layers,
                            int32_t n_layers, int32_t pos0, float* hidden, int32_t T, char* err,
                            int32_t errlen);
void cake_engine_drop_session(void* engine, uint64_t session);
// [rank, world, first layer, end layer]
int32_t cake_engine_rank_info(void* engine, int32_t* out4);
// [V, H, L, nh, nkv, hd, I, max_seq]
int32_t cake_engine_info(void* engine, int32_t* out8);
// EOS ids of the config (up to cap); returns the count
int32_t cake_engine_eos(void* engine, int32_t* out, int32_t cap);
// Prefill `prompt` from position 0, then generate up to max_new tokens (the first comes
// from the prefill logits), stopping after an EOS id.  Tokens go to out[] (and cb).
// Returns 0 or an error code (message in err).
int32_t cake_engine_generate(void* engine, const int32_t* prompt, int32_t n_prompt,
                             int32_t max_new, const struct CakeEngineSampling* sampling,
                             const int32_t* eos, int32_t n_eos, cake_engine_token_cb cb,
                             void* ctx, int32_t* out, int32_t out_cap,
                             struct CakeEngineStats* stats, char* err, int32_t errlen);
// Continue the last generation for up to max_new more tokens (same sampling, the device
// state where the previous generate / continue left it, EOS included): chat turns that
// extend a context, and benchmarks that time exactly max_new decode steps.
int32_t cake_engine_continue(void* engine, int32_t max_new, const int32_t* eos, int32_t n_eos,
                             cake_engine_token_cb cb, void* ctx, int32_t* out, int32_t out_cap,
                             struct CakeEngineStats* stats, char* err, int32_t errlen);
// Teacher forcing (tests): prefill `prompt`, then one decode step per forced token (the
// decode kernels, hops and all-reduces, launched eagerly); out[(n_forced + 1) x V] = the
// f32 logits after the prompt and after each forced token.  Rank 0 of any mode.
int32_t cake_engine_forced_logits(void* engine, const int32_t* prompt, int32_t n_prompt,
                                  const int32_t* forced, int32_t n_forced, float* out, char* err,
                                  int32_t errlen);
// "rank:first-last,..." layer runs of the token's walk (placement check); bytes written.
int32_t cake_engine_walk(void* engine, char* out, int32_t cap);
// Logits of the last prompt position after a prefill only (f32 [V] to host), for tests.
int32_t cake_engine_prefill_logits(void* engine, const int32_t* prompt, int32_t n_prompt,
                                   float* out, char* err, int32_t errlen);
void cake_engine_close(void* engine);

#ifdef __cplusplus
}
#endif
