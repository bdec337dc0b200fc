#include "proto.h"

#include <cstring>
#include <stdexcept>

namespace cake {

namespace {

struct W {
  std::string out;
  void u32(uint32_t v) {
    for (int i = 3; i >= 0; --i) out += (char)((v >> (8 * i)) & 0xff);
  }
  void u64(uint64_t v) {
    for (int i = 7; i >= 0; --i) out += (char)((v >> (8 * i)) & 0xff);
  }
  void bytes(const uint8_t* p, uint64_t n) {
    if (n > 0xffffffffull) throw std::runtime_error("proto: vector too long");
    u32((uint32_t)n);
    out.append(reinterpret_cast<const char*>(p), (size_t)n);
  }
  void str(const std::string& s) { bytes(reinterpret_cast<const uint8_t*>(s.data()), s.size()); }
  void tensor(const RawTensor& t) {
    bytes(t.data, t.nbytes);
    str(t.dtype);
    u32((uint32_t)t.shape.size());
    for (uint64_t d : t.shape) u64(d);
  }
};

struct R {
  const uint8_t* p;
  const uint8_t* end;
  void need(size_t n) {
    if ((size_t)(end - p) < n) throw std::runtime_error("proto: truncated message");
  }
  uint32_t u32() {
    need(4);
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) v = (v << 8) | p[i];
    p += 4;
    return v;
  }
  uint64_t u64() {
    need(8);
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    p += 8;
    return v;
  }
  std::string str() {
    uint32_t n = u32();
    need(n);
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  RawTensor tensor() {
    RawTensor t;
    t.nbytes = u32();
    need(t.nbytes);
    t.data = p;
    p += t.nbytes;
    t.dtype = str();
    uint32_t nd = u32();
    for (uint32_t i = 0; i < nd; ++i) t.shape.push_back(u64());
    return t;
  }
};

}  // namespace

std::string encode_body(const Message& m) {
  W w;
  w.u32((uint32_t)m.type);
  switch (m.type) {
    case MsgType::Hello:
    case MsgType::Ping:
    case MsgType::Pong:
      break;
    case MsgType::WorkerInfo:
      w.str(m.info.version);
      w.str(m.info.dtype);
      w.str(m.info.os);
      w.str(m.info.arch);
      w.str(m.info.device);
      w.u64(m.info.device_idx);
      w.u64(m.info.latency_hi);
      w.u64(m.info.latency_lo);
      break;
    case MsgType::SingleOp:
      w.str(m.layer_name);
      w.tensor(m.x);
      w.u64(m.index_pos);
      w.u64(m.block_idx);
      break;
    case MsgType::Batch:
      w.tensor(m.x);
      w.u32((uint32_t)m.batch.size());
      for (const auto& b : m.batch) {
        w.str(b.layer_name);
        w.u64(b.index_pos);
        w.u64(b.block_idx);
      }
      break;
    case MsgType::Tensor:
      w.tensor(m.x);
      break;
    case MsgType::Reset:
      w.u64(m.session);
      break;
    case MsgType::Error:
      w.str(m.error);
      break;
    default:
      throw std::runtime_error("proto: unknown message type");
  }
  if (w.out.size() > kMaxMessageSize) throw std::runtime_error("proto: message too large");
  return std::move(w.out);
}

Message decode_body(const uint8_t* body, size_t n) {
  R r{body, body + n};
  Message m;
  const uint32_t tag = r.u32();
  if (tag > (uint32_t)MsgType::Pong) throw std::runtime_error("proto: unknown message tag " + std::to_string(tag));
  m.type = (MsgType)tag;
  switch (m.type) {
    case MsgType::Hello:
    case MsgType::Ping:
    case MsgType::Pong:
      break;
    case MsgType::WorkerInfo:
      m.info.version = r.str();
      m.info.dtype = r.str();
      m.info.os = r.str();
      m.info.arch = r.str();
      m.info.device = r.str();
      m.info.device_idx = r.u64();
      m.info.latency_hi = r.u64();
      m.info.latency_lo = r.u64();
      break;
    case MsgType::SingleOp:
      m.layer_name = r.str();
      m.x = r.tensor();
      m.index_pos = r.u64();
      m.block_idx = r.u64();
      break;
    case MsgType::Batch: {
      m.x = r.tensor();
      const uint32_t nb = r.u32();
      for (uint32_t i = 0; i < nb; ++i) {
        BatchItem b;
        b.layer_name = r.str();
        b.index_pos = r.u64();
        b.block_idx = r.u64();
        m.batch.push_back(std::move(b));
      }
      break;
    }
    case MsgType::Tensor:
      m.x = r.tensor();
      break;
    case MsgType::Reset:
      m.session = r.u64();
      break;
    case MsgType::Error:
      m.error = r.str();
      break;
  }
  if (r.p != r.end) throw std::runtime_error("proto: trailing bytes in message");
  return m;
}

void encode_header(uint32_t n, uint8_t out[8]) {
  if (n > kMaxMessageSize) throw std::runtime_error("proto: message too large");
  // little-endian on the wire (the reference's double swap, Appendix A)
  for (int i = 0; i < 4; ++i) out[i] = (uint8_t)((kProtoMagic >> (8 * i)) & 0xff);
  for (int i = 0; i < 4; ++i) out[4 + i] = (uint8_t)((n >> (8 * i)) & 0xff);
}

uint32_t decode_header(const uint8_t in[8]) {
  uint32_t magic = 0, n = 0;
  for (int i = 3; i >= 0; --i) magic = (magic << 8) | in[i];
  for (int i = 3; i >= 0; --i) n = (n << 8) | in[4 + i];
  if (magic != kProtoMagic) throw std::runtime_error("proto: bad magic");
  if (n > kMaxMessageSize) throw std::runtime_error("proto: message too large");
  return n;
}

}  // namespace cake
