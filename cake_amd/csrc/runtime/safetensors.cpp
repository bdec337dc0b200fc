#include "safetensors.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace cake {

uint64_t dtype_size(const std::string& d) {
  if (d == "F64" || d == "I64" || d == "U64") return 8;
  if (d == "F32" || d == "I32" || d == "U32") return 4;
  if (d == "F16" || d == "BF16" || d == "I16" || d == "U16") return 2;
  if (d == "I8" || d == "U8" || d == "BOOL" || d == "F8_E4M3" || d == "F8_E5M2") return 1;
  throw std::runtime_error("safetensors: unknown dtype " + d);
}

SafeTensorsFile::SafeTensorsFile(const std::string& path) : path_(path) {
  fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd_ < 0) throw std::runtime_error("can't open " + path + ": " + std::strerror(errno));
  struct stat st {};
  if (fstat(fd_, &st) != 0) throw std::runtime_error("can't stat " + path);
  size_ = (uint64_t)st.st_size;
  if (size_ < 8) throw std::runtime_error(path + ": not a safetensors file");
  void* m = ::mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0);
  if (m == MAP_FAILED) throw std::runtime_error("mmap " + path + ": " + std::strerror(errno));
  base_ = static_cast<uint8_t*>(m);
  uint64_t n = 0;
  for (int i = 7; i >= 0; --i) n = (n << 8) | base_[i];
  if (n > size_ - 8 || n > (100ull << 20)) throw std::runtime_error(path + ": bad header length");
  const Json hdr = Json::parse(std::string(reinterpret_cast<const char*>(base_ + 8), n));
  const uint64_t data0 = 8 + n;
  for (const auto& kv : hdr.members()) {
    if (kv.first == "__metadata__") {
      for (const auto& m2 : kv.second.members())
        if (m2.second.is_string()) metadata_[m2.first] = m2.second.as_string();
      continue;
    }
    TensorView v;
    v.name = kv.first;
    v.dtype = kv.second.get("dtype").as_string();
    // every header integer is validated before use: negative values and
    // overflowing products are rejected (a crafted header must not produce a
    // view outside the mapping)
    const auto bad = [&](const char* what) {
      return std::runtime_error(path + ": tensor " + v.name + " " + what);
    };
    uint64_t numel = 1;
    for (const auto& d : kv.second.get("shape").items()) {
      const int64_t dim = d.as_int();
      if (dim < 0) throw bad("has a negative dimension");
      if (dim != 0 && numel > UINT64_MAX / (uint64_t)dim) throw bad("shape overflows");
      v.shape.push_back((uint64_t)dim);
      numel *= (uint64_t)dim;
    }
    const auto& off = kv.second.get("data_offsets");
    const int64_t bi = off.at(0).as_int(), ei = off.at(1).as_int();
    if (bi < 0 || ei < 0) throw bad("has negative data offsets");
    const uint64_t b = (uint64_t)bi, e = (uint64_t)ei;
    if (e < b || e > size_ - data0) throw bad("out of bounds");
    const uint64_t es = dtype_size(v.dtype);
    if (es != 0 && numel > UINT64_MAX / es) throw bad("byte size overflows");
    if (e - b != numel * es) throw bad("size mismatch");
    v.offset = data0 + b;
    v.data = base_ + v.offset;
    v.nbytes = e - b;
    names_.push_back(v.name);
    views_.emplace(v.name, std::move(v));
  }
}

SafeTensorsFile::~SafeTensorsFile() {
  if (base_) ::munmap(base_, size_);
  if (fd_ >= 0) ::close(fd_);
}

const TensorView& SafeTensorsFile::tensor(const std::string& n) const {
  auto it = views_.find(n);
  if (it == views_.end()) throw std::out_of_range("tensor not found: " + n);
  return it->second;
}

void write_safetensors(const std::string& path, const std::vector<TensorToWrite>& tensors,
                       const std::map<std::string, std::string>& metadata) {
  Json hdr = Json::object();
  if (!metadata.empty()) {
    Json m = Json::object();
    for (const auto& kv : metadata) m.set(kv.first, Json::string(kv.second));
    hdr.set("__metadata__", std::move(m));
  }
  uint64_t off = 0;
  for (const auto& t : tensors) {
    uint64_t numel = 1;
    Json shape = Json::array();
    for (uint64_t d : t.shape) {
      shape.push(Json::integer((int64_t)d));
      numel *= d;
    }
    if (numel * dtype_size(t.dtype) != t.nbytes)
      throw std::runtime_error("write_safetensors: " + t.name + " byte size mismatch");
    Json e = Json::object();
    e.set("dtype", Json::string(t.dtype));
    e.set("shape", std::move(shape));
    Json offs = Json::array();
    offs.push(Json::integer((int64_t)off));
    offs.push(Json::integer((int64_t)(off + t.nbytes)));
    e.set("data_offsets", std::move(offs));
    hdr.set(t.name, std::move(e));
    off += t.nbytes;
  }
  std::string h = hdr.dump();
  while ((8 + h.size()) % 8) h += ' ';  // align the data section
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("can't write " + tmp);
  uint8_t len[8];
  uint64_t n = h.size();
  for (int i = 0; i < 8; ++i) len[i] = (uint8_t)((n >> (8 * i)) & 0xff);
  bool ok = std::fwrite(len, 1, 8, f) == 8 && std::fwrite(h.data(), 1, h.size(), f) == h.size();
  for (const auto& t : tensors)
    ok = ok && (t.nbytes == 0 || std::fwrite(t.data, 1, t.nbytes, f) == t.nbytes);
  ok = (std::fclose(f) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0)
    throw std::runtime_error("failed writing " + path);
}

std::map<std::string, std::string> load_weight_map(const std::string& dir) {
  std::map<std::string, std::string> wm;
  const std::string idx = dir + "/model.safetensors.index.json";
  std::ifstream f(idx);
  if (f) {
    std::stringstream ss;
    ss << f.rdbuf();
    const Json j = Json::parse(ss.str());
    for (const auto& kv : j.get("weight_map").members()) wm[kv.first] = kv.second.as_string();
    return wm;
  }
  const std::string single = dir + "/model.safetensors";
  SafeTensorsFile st(single);
  for (const auto& n : st.names()) wm[n] = "model.safetensors";
  return wm;
}

Checkpoint::Checkpoint(const std::string& dir) : dir_(dir), weight_map_(load_weight_map(dir)) {}

const TensorView& Checkpoint::tensor(const std::string& name) {
  auto it = weight_map_.find(name);
  if (it == weight_map_.end()) throw std::out_of_range("tensor not in checkpoint: " + name);
  auto& f = files_[it->second];
  if (!f) f = std::make_unique<SafeTensorsFile>(dir_ + "/" + it->second);
  return f->tensor(name);
}

}  // namespace cake
