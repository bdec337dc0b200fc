// Native decode driver: the per-token host loop of every serving mode.
//
// Replaces the reference master's token loop (cake-core/src/cake/master.rs:80-124:
// `next_token` per step, tok/s timer restarted after the first token) and the
// generator's per-step forward + sample (cake-core/src/models/llama3/llama.rs:277-341).
// Here one decode step (every layer, the head and the token choice, plus the
// device-side pipeline hops / all-reduces of a multi-rank engine) is ONE captured
// hipGraph, and the chosen token never leaves the device except for reporting.
// What is left for the host is this loop, in C++ with the Python GIL released:
//
//   * replay the step graph whose decode-attention split cap covers the live
//     length (one graph per position bucket, chosen through a host table),
//   * copy the replay's k tokens from the device history into a pinned ring and
//     record an event — and only then wait for the PREVIOUS replay's event, so
//     the GPU always has the next step queued while the host reads one back,
//   * stop at EOS, at n tokens, or when the per-token callback asks (streaming
//     API clients), and report per-token device time (p50/p99: BASELINE.md §2).
//
// A worker rank of a pipeline / tensor-parallel engine passes no history and no
// callbacks: its replays are enqueued at once and paced by the device-side receives.
// An optional `announce` callback runs one chunk of replays ahead of them (the
// master's control message telling the workers how many replays to enqueue).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>
#include <vector>

#define CAKE_API extern "C" __attribute__((visibility("default")))

#include "graph_loop.h"

namespace {

// The read-back ring (pinned host slots) and the replay events persist per thread and
// device: allocating them per call put a pinned allocation, its free (which can wait on
// the device) and four event creations inside every generate call — ~0.5 ms, 1 % of a
// 20-token run.  Never freed (process lifetime; freeing at thread exit could run after
// the HIP runtime is gone).
struct Ring {
  int32_t* host = nullptr;
  int cap = 0;  // int32 slots
  int dev = -1;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
};
thread_local Ring t_ring;

hipError_t ring_for(int slots, Ring*& out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  Ring& r = t_ring;
  if (r.dev != dev) {  // events belong to a device: (re)create them there
    for (auto& ev : r.ev) {
      if (ev) (void)hipEventDestroy(ev);
      ev = nullptr;
      if ((e = hipEventCreate(&ev)) != hipSuccess) return e;
    }
    r.dev = dev;
  }
  if (r.cap < slots) {
    if (r.host) (void)hipHostFree(r.host);
    r.host = nullptr;
    r.cap = 0;
    if ((e = hipHostMalloc((void**)&r.host, sizeof(int32_t) * slots, hipHostMallocDefault)) !=
        hipSuccess)
      return e;
    r.cap = slots;
  }
  out = &r;
  return hipSuccess;
}

inline int fail(hipError_t e) { return (int)e; }

}  // namespace

#define CAKE_TRY(x)                              \
  do {                                           \
    const hipError_t e_ = (x);                   \
    if (e_ != hipSuccess) return fail(e_);       \
  } while (0)

CAKE_API int cake_graph_decode(const CakeLoopSpec* s, CakeLoopResult* r) {
  if (!s || !r || s->n_execs <= 0 || !s->execs || s->k <= 0 || s->n < 0 || !s->bucket_of ||
      s->n_len <= 0)
    return (int)hipErrorInvalidValue;
  *r = CakeLoopResult{0, 0, s->pos, 0, 0.0};
  if (s->n == 0) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  hipStream_t st = (hipStream_t)s->stream;
  const int k = s->k;
  const int replays = (s->n + k - 1) / k;
  const bool readback = s->hist != nullptr;
  if (readback && (!s->out_tokens || s->out_cap < s->n)) return (int)hipErrorInvalidValue;
  const int chunk = s->chunk > 0 ? s->chunk : replays;
  int pos = s->pos;
  // one replay of the graph whose attention split cap covers the live length at its
  // last step (+1: room for a pushed token)
  auto launch = [&]() -> hipError_t {
    int len = pos + k + 1;
    if (len >= s->n_len) len = s->n_len - 1;
    int b = s->bucket_of[len];
    if (b < 0 || b >= s->n_execs) b = s->n_execs - 1;
    pos += k;
    return hipGraphLaunch((hipGraphExec_t)s->execs[b], st);
  };
  if (!readback && !s->on_token && !s->announce) {
    // worker rank: enqueue every replay and return at once (the device-side
    // receives pace them; the host goes back to its control channel)
    for (int i = 0; i < replays; ++i) CAKE_TRY(launch());
    r->replays = replays;
    r->pos = pos;
    return 0;
  }

  // two ring slots of k tokens (replay p+1 fills one while p is read from the
  // other); three replay events (p+1 is recorded while p-1's still bounds p's
  // interval) and a start event
  Ring* rp = nullptr;
  CAKE_TRY(ring_for(2 * k, rp));
  Ring& ring = *rp;
  CAKE_TRY(hipEventRecord(ring.ev[3], st));
  hipEvent_t prev_done = ring.ev[3];

  int issued = 0;          // replays enqueued
  int announced = 0;       // replays announced to the workers
  int pending = -1;        // replay index waiting for read-back
  bool stop = false;
  hipError_t err = hipSuccess;  // first failure inside the loop (cleanup below)
#define CAKE_LOOP_TRY(x)            \
  do {                              \
    const hipError_t e_ = (x);      \
    if (e_ != hipSuccess) {         \
      err = e_;                     \
      goto loop_end;                \
    }                               \
  } while (0)
  while (!stop) {
    int cur = -1;
    if (issued < replays) {
      // keep the announcements one chunk ahead of the replays, so the workers have
      // the next chunk enqueued before the master reaches it
      while (s->announce && announced < replays && announced - issued <= chunk) {
        const int c = chunk < replays - announced ? chunk : replays - announced;
        if (s->announce(s->announce_ctx, announced, c) != 0) CAKE_LOOP_TRY(hipErrorUnknown);
        announced += c;
      }
      CAKE_LOOP_TRY(launch());
      const int slot = issued & 1;
      if (readback) {
        const int lo = s->base + issued * k;
        CAKE_LOOP_TRY(hipMemcpyAsync(ring.host + slot * k, s->hist + lo, sizeof(int32_t) * k,
                                     hipMemcpyDeviceToHost, st));
      }
      CAKE_LOOP_TRY(hipEventRecord(ring.ev[issued % 3], st));
      cur = issued++;
    }
    if (pending >= 0) {
      const int slot = pending & 1;
      hipEvent_t done = ring.ev[pending % 3];
      CAKE_LOOP_TRY(hipEventSynchronize(done));
      float ms = 0.f;
      CAKE_LOOP_TRY(hipEventElapsedTime(&ms, prev_done, done));
      ms /= (float)k;
      const int have = s->n - pending * k;
      const int m = have < k ? have : k;
      for (int i = 0; i < m && !stop; ++i) {
        const int idx = r->n_tokens;
        if (idx < s->out_cap && s->out_ms) s->out_ms[idx] = ms;
        if (readback) {
          const int32_t tok = ring.host[slot * k + i];
          s->out_tokens[idx] = tok;
          r->n_tokens = idx + 1;
          if (s->on_token && s->on_token(s->token_ctx, tok) != 0) stop = true;
          for (int e = 0; e < s->n_eos && !stop; ++e)
            if (s->eos[e] == tok) stop = true;
        } else {
          r->n_tokens = idx + 1;
        }
      }
      prev_done = done;  // the next replay's interval starts where this one ended
    }
    pending = cur;
    if (pending < 0) break;
  }
loop_end:
#undef CAKE_LOOP_TRY
  // replays announced to the workers but not yet issued (a stop inside an announced
  // chunk, or an error) still run, unread: every rank must replay the same number of
  // hops, or the workers wait in device-side receives until their hop timeout.  Then
  // drain the stream before returning, so no read-back into the thread-local pinned
  // ring is still in flight when the next call reuses it.
  for (; issued < announced; ++issued) {
    const hipError_t e = launch();
    if (e != hipSuccess) {
      if (err == hipSuccess) err = e;
      break;
    }
  }
  {
    const hipError_t e = hipStreamSynchronize(st);
    if (err == hipSuccess) err = e;
  }
  if (err != hipSuccess) return fail(err);
  r->replays = issued;
  r->pos = pos;
  r->stopped = stop ? 1 : 0;
  r->wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}
