// cake wire protocol codec (byte-compatible with the reference).
//
// Frame (cake-core/src/cake/proto/message.rs:83-97,138-176; proto/mod.rs:4,7):
//   u32 MAGIC 0x0104F4C7 | u32 SIZE | body, SIZE <= 512 MiB.
// The reference writes the header with tokio's big-endian write_u32 of an
// already byte-swapped value, so on little-endian hosts MAGIC and SIZE are
// LITTLE-endian on the wire.  The body is a speedy
// BigEndian encoding: enum tag u32, String/Vec = u32 length + elements,
// usize = u64, u128 = 16 bytes.
//
// Variants 0-4 are the reference's (Hello, WorkerInfo, SingleOp, Batch,
// Tensor).  Extensions (a reference peer never sends them): 5 Reset (clear
// the connection's KV — fixes Appendix E Q7), 6 Error (worker-side failure
// instead of aborting, Q6), 7 Ping / 8 Pong (liveness).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace cake {

constexpr uint32_t kProtoMagic = 0x0104F4C7u;
constexpr uint32_t kMaxMessageSize = 512u * 1024u * 1024u;

enum class MsgType : uint32_t {
  Hello = 0, WorkerInfo = 1, SingleOp = 2, Batch = 3, Tensor = 4,
  Reset = 5, Error = 6, Ping = 7, Pong = 8,
};

struct RawTensor {
  std::string dtype;            // candle names: "f16", "bf16", "f32", "u32", ...
  std::vector<uint64_t> shape;
  const uint8_t* data = nullptr;  // view (encode input / decode output into the frame)
  uint64_t nbytes = 0;
};

struct WorkerInfo {
  std::string version, dtype, os, arch, device;
  uint64_t device_idx = 0;
  uint64_t latency_hi = 0, latency_lo = 0;  // u128 milliseconds
};

struct BatchItem {
  std::string layer_name;
  uint64_t index_pos = 0, block_idx = 0;
};

struct Message {
  MsgType type = MsgType::Hello;
  WorkerInfo info;
  std::string layer_name;     // SingleOp
  RawTensor x;                // SingleOp / Batch / Tensor
  uint64_t index_pos = 0, block_idx = 0;
  std::vector<BatchItem> batch;
  std::string error;          // Error
  uint64_t session = 0;       // Reset
};

// body only (no frame header)
std::string encode_body(const Message& m);
// `body` must outlive the returned message (x.data points into it)
Message decode_body(const uint8_t* body, size_t n);

// 8-byte frame header for a body of n bytes
void encode_header(uint32_t n, uint8_t out[8]);
// returns body size; throws on bad magic / oversize
uint32_t decode_header(const uint8_t in[8]);

}  // namespace cake
