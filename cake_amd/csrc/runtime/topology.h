// topology.yml: worker name -> {host, description?, layers[]}.
//
// Semantics of cake-core/src/cake/topology.rs:
//   * range expansion `prefix.A-B` (inclusive; error unless B > A) with the
//     regex ^(.+[^\d])(\d+)-(\d+)$, only for text models (topology.rs:9-11,47-76);
//   * get_node_for_layer: exact layer-name match (topology.rs:81-92) — here the
//     first match in FILE order (deterministic, unlike the reference HashMap);
//   * is_text_model_layer_owner: tensor name starts with "{layer}." (topology.rs:23-35).
// The parser accepts the YAML subset topology files use: nested block
// mappings, block ("- x") and flow ("[a, b]") sequences, quoted/plain
// scalars, comments, and an empty document / "{}" (= everything local).
#pragma once

#include <string>
#include <vector>

namespace cake {

struct TopoNode {
  std::string name;
  std::string host;
  std::string description;
  bool has_description = false;
  std::vector<std::string> layers;

  bool is_text_model_layer_owner(const std::string& full_name) const;
};

struct Topology {
  std::vector<TopoNode> nodes;

  static Topology parse(const std::string& yaml, bool text_model);
  static Topology from_path(const std::string& path, bool text_model);
  const TopoNode* node_for_layer(const std::string& layer) const;
  const TopoNode* find(const std::string& name) const;
  std::string to_yaml() const;
};

// Expand "prefix.A-B" into prefix.A .. prefix.B; throws on B <= A.
std::vector<std::string> expand_layer_range(const std::string& spec);

}  // namespace cake
