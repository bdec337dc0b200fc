// Native Stable Diffusion engine (libcake_engine.so): the whole image generation —
// text encoders, the classifier-free-guided denoising loop with its scheduler, the VAE
// decode — as host C++ over the gfx950 kernels' C entry points, with no interpreter.
//
// What it replaces: the reference's native SD pipeline (cake-core/src/models/sd/sd.rs:
// 320-532 generate_image, unet.rs:43-100, vae.rs:55-108, clip.rs:24-75 over candle) and
// this repo's Python host loop (models/sd/pipeline.py, unet.py, vae.py, clip.py), whose
// kernels and launch order it reproduces.  Tokenization stays with the caller (the HF
// tokenizers library, as for the native Llama engine): the engine takes padded CLIP ids.
//
// Device path per generation:
//   * text: CLIP-L (and OpenCLIP-bigG for xl / turbo) over the [uncond; cond] ids ->
//     the [2, 77, D] context (both encoders concatenated on the feature axis);
//     every cross-attention's k|v projection of it computed once into persistent buffers;
//   * denoise: the first step eagerly (convolution autotuning, GEMM plans), every later
//     step ONE hipGraph replay: time embedding from the device timestep table -> UNet
//     (NHWC, fused epilogues) -> CFG combine + scheduler update + next input
//     (sched_step) -> step += 1;
//   * decode: latents / vae_scale -> VAE decoder -> RGB8 on the device.
#pragma once

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct CakeSdOpts {
  const char* version;   // "v1-5" | "v2-1" | "xl" | "turbo" (null: cake_sd.json / "v1-5")
  int32_t width;         // 0: the version's default
  int32_t height;
  int32_t dtype;         // 0 bf16, 1 f16
  int32_t device;
  int32_t init;          // 1: seeded random weights (no component file is read)
  int32_t autotune;      // 1: time the convolution variants on the first step (else planner)
  int32_t tiny;          // 1: the small test architecture (models/sd/config.py tiny_config)
  uint64_t seed;         // random-init seed
  // component files (null: resolved under the model directory, weights.py COMPONENT_FILES)
  const char* unet_path;
  const char* vae_path;
  const char* clip_path;
  const char* clip2_path;
  int32_t parts;         // components to load: 1 unet | 2 vae | 4 clip | 8 clip2 (0: all)
  // components served by TCP workers ("host:port", the reference's topology: a worker's
  // SingleOp "unet" / "vae" / "clip" / "clip2"; null = local).  A remote UNet runs every
  // step as one round trip (no step graph); generate() needs each component local or
  // remote.
  const char* remote_unet;
  const char* remote_vae;
  const char* remote_clip;
  const char* remote_clip2;
  double remote_timeout_s;  // per request (0: 120)
} CakeSdOpts;

typedef struct CakeSdGenArgs {
  const int32_t* cond;      // [77] ids of the first tokenizer
  const int32_t* uncond;    // [77] or null: no classifier-free guidance
  const int32_t* cond2;     // [77] ids of the second tokenizer (xl / turbo)
  const int32_t* uncond2;
  int32_t n_steps;
  float guidance;
  uint64_t seed;            // the ancestral-noise key (sched_step), and the latent noise
                            // when init_noise is null
  const float* init_noise;  // optional [4 * (h/8) * (w/8)] standard-normal latent noise
  int32_t use_graph;        // 1: every step after the first is one hipGraph replay
  // img2img: the schedule's steps from t_start on, starting from init_latents ([bsize] x the
  // encoded image, scaled and noised to ts[t_start] by the caller); null = txt2img
  int32_t t_start;
  const float* init_latents;
  // images per sample (the reference's bsize): the UNet runs 2 bsize rows under guidance,
  // the text rows repeated [uncond, cond] x bsize as the reference's
  // text_embeddings.repeat((bsize, 1, 1)); init_noise then holds bsize latents, rgb /
  // latents_out bsize images (img2img: init_latents bsize latents).  0 = 1.
  int32_t bsize;
  // intermediary images: every step index i (of the full schedule) with i % intermediary
  // == 0 is decoded and handed to on_image(cb_ctx, i, bsize, rgb [bsize, height, width, 3])
  // before the next step runs (0 / null: none)
  int32_t intermediary;
  void (*on_image)(void* cb_ctx, int32_t step, int32_t n_images, const uint8_t* rgb);
  void* cb_ctx;
} CakeSdGenArgs;

typedef struct CakeSdResult {
  int32_t width, height, n_steps;
  double text_s, denoise_s, vae_s;
} CakeSdResult;

// Open (load or random-init) every component; null + err on failure.
void* cake_sd_open(const char* model_dir, const CakeSdOpts* opts, char* err, int32_t errlen);

// Split UNet over one process per GPU (BASELINE config 5; the reference reaches a remote
// UNet once per step: cake-core/src/models/sd/sd.rs:464-513, unet.rs:81-100).  The UNet's
// stages (down.i, mid, up.i) run in contiguous runs over ranks 0 .. used-1 (rank 0 first;
// `owners`, if given, names the rank of every stage and must be such runs).  Each denoise
// step is one graph replay per rank: bulk device hops (hop.hip, IPC-mapped uncached inboxes)
// carry the feature map to the next run's rank, every skip tensor once from the rank that
// pushes it straight to the rank whose up stage pops it, and the prediction back to rank
// 0, which runs the text encoders, the scheduler and the VAE.  Control plane (IPC
// handles, the generation's timesteps and text context) over TCP to rank 0 at
// master_addr.  Rank 0 generates with cake_sd_generate; the others call cake_sd_serve.
typedef struct CakeSdSplitOpts {
  int32_t rank, world;
  const char* master_addr;   // "host:port" rank 0 listens on
  double timeout_s;          // a hop wait bound (the error word instead of a hang)
  double connect_timeout_s;  // ranks > 0: how long to retry reaching rank 0
  const int32_t* owners;     // [n_owners == the UNet's stage count] or null (even split)
  int32_t n_owners;
} CakeSdSplitOpts;
void* cake_sd_open_split(const char* model_dir, const CakeSdOpts* opts,
                         const CakeSdSplitOpts* split, char* err, int32_t errlen);
// ranks > 0: serve rank 0's generations until it closes the group
int32_t cake_sd_serve(void* engine, char* err, int32_t errlen);
// (rank, world, stages, ranks used, first stage of this rank, end stage) of an engine
void cake_sd_split_info(void* engine, int32_t* out6);
// One sample of bsize images: rgb [bsize * height * width * 3] u8; latents_out (optional)
// [bsize * 4 * h/8 * w/8] f32 (the final latents); step_s (optional) [n_steps] seconds per
// step (device time).
int32_t cake_sd_generate(void* engine, const CakeSdGenArgs* args, uint8_t* rgb,
                         float* latents_out, double* step_s, CakeSdResult* result, char* err,
                         int32_t errlen);
void cake_sd_close(void* engine);
// (width, height, context dim, model dtype, text dim 1, text dim 2 or 0) of an open engine
void cake_sd_info(void* engine, int32_t* out6);

// Component entry points (tests / parity checks; f32 host tensors in and out):
// which = 0 CLIP (first encoder), 1 the second encoder; ids [B, 77] -> out [B, 77, D].
int32_t cake_sd_text(void* engine, int32_t which, const int32_t* ids, int32_t B, float* out,
                     char* err, int32_t errlen);
// One eager UNet forward: sample [B, 4, h, w] (NCHW), timestep t, context [B, 77, Dctx]
// -> out [B, 4, h, w].
int32_t cake_sd_unet(void* engine, const float* sample, int32_t B, float t, const float* ctx,
                     float* out, char* err, int32_t errlen);
// VAE decode of z [1, 4, h, w] (already divided by vae_scale) -> image [1, 3, H, W] in [-1, 1].
int32_t cake_sd_vae_decode(void* engine, const float* z, float* img, char* err, int32_t errlen);
// VAE encode of an image [1, 3, H, W] in [-1, 1] -> the posterior moments [1, 8, h, w]
// (mean | logvar; the caller samples, as vae.py AutoencoderKL.encode does).
int32_t cake_sd_vae_encode(void* engine, const float* img, float* moments, char* err,
                           int32_t errlen);
// img2img with the topology's VAE worker: the image [1, 3, H, W] -> the latent sample
// [1, 4, h, w] drawn by the worker (SingleOp "vae" on pack([1, img])).  With a remote VAE,
// cake_sd_vae_decode goes to the worker as well.
int32_t cake_sd_vae_encode_remote(void* engine, const float* img, float* sample, char* err,
                                  int32_t errlen);

#ifdef __cplusplus
}
#endif
