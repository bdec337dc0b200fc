// safetensors reader (mmap) / writer and HF sharded-index handling.
//
// Reference: candle VarBuilder::from_mmaped_safetensors over the shard list of
// model.safetensors.index.json (cake-core/src/utils/mod.rs:32-104) and the
// split tool's re-serialisation (cake-split-model/src/main.rs:105-220).
// Format: u64 LE header length N | N bytes JSON {name: {dtype, shape,
// data_offsets:[b,e]}, "__metadata__"?: {str: str}} | data (offsets relative
// to 8 + N).  Readers here never copy: tensors are views into the mapping, so
// a rank uploads only the tensors it owns straight from the page cache.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "json.h"

namespace cake {

struct TensorView {
  std::string name, dtype;
  std::vector<uint64_t> shape;
  const uint8_t* data = nullptr;
  uint64_t nbytes = 0;
  uint64_t offset = 0;  // absolute file offset of the data
};

class SafeTensorsFile {
 public:
  explicit SafeTensorsFile(const std::string& path);
  ~SafeTensorsFile();
  SafeTensorsFile(const SafeTensorsFile&) = delete;
  SafeTensorsFile& operator=(const SafeTensorsFile&) = delete;

  const std::string& path() const { return path_; }
  const std::vector<std::string>& names() const { return names_; }
  bool has(const std::string& n) const { return views_.count(n) != 0; }
  const TensorView& tensor(const std::string& n) const;
  const std::map<std::string, std::string>& metadata() const { return metadata_; }
  const uint8_t* base() const { return base_; }
  uint64_t size() const { return size_; }

 private:
  std::string path_;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  uint64_t size_ = 0;
  std::vector<std::string> names_;
  std::map<std::string, TensorView> views_;
  std::map<std::string, std::string> metadata_;
};

struct TensorToWrite {
  std::string name, dtype;
  std::vector<uint64_t> shape;
  const uint8_t* data;
  uint64_t nbytes;
};

uint64_t dtype_size(const std::string& dtype);
void write_safetensors(const std::string& path, const std::vector<TensorToWrite>& tensors,
                       const std::map<std::string, std::string>& metadata = {});

// weight_map of <dir>/model.safetensors.index.json, or every tensor of
// <dir>/model.safetensors when no index exists (utils/mod.rs:32-82).
std::map<std::string, std::string> load_weight_map(const std::string& dir);

// Lazily opened shards of a checkpoint directory.
class Checkpoint {
 public:
  explicit Checkpoint(const std::string& dir);
  const TensorView& tensor(const std::string& name);
  bool has(const std::string& name) const { return weight_map_.count(name) != 0; }
  const std::map<std::string, std::string>& weight_map() const { return weight_map_; }

 private:
  std::string dir_;
  std::map<std::string, std::string> weight_map_;
  std::map<std::string, std::unique_ptr<SafeTensorsFile>> files_;
};

}  // namespace cake
