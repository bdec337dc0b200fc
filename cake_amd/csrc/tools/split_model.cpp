// cake-split-model: extract per-worker weight bundles from a sharded HF checkpoint.
//
// Behaviour of cake-split-model/src/main.rs:141-222: for every worker of the
// topology (or --worker NAME), keep the tensors whose name starts with
// "{layer}." for one of its layers, write
//   <output>/<worker>-node/model/{model.safetensors.index.json, reduced.safetensors}
//   <output>/<worker>-node/topology.yml   (only this worker)
// and re-open the result as a sanity check.  Additions: config.json (and
// tokenizer files when present) are copied into the bundle so a worker can
// start from it alone, and tensors are copied straight from the mmapped shards.
#include <sys/stat.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "json.h"
#include "safetensors.h"
#include "topology.h"

using namespace cake;

static void mkdirs(const std::string& p) {
  std::string cur;
  for (size_t i = 0; i < p.size(); ++i) {
    cur += p[i];
    if (p[i] == '/' || i + 1 == p.size()) ::mkdir(cur.c_str(), 0755);
  }
}

static bool exists(const std::string& p) {
  struct stat st {};
  return ::stat(p.c_str(), &st) == 0;
}

static void copy_file(const std::string& a, const std::string& b) {
  std::ifstream in(a, std::ios::binary);
  std::ofstream out(b, std::ios::binary);
  out << in.rdbuf();
}

static void usage() {
  std::cerr << "usage: cake-split-model --model-path DIR --topology FILE --output DIR [--worker NAME]\n";
}

int main(int argc, char** argv) {
  std::string model_path = "./cake-data/Meta-Llama-3-8B/", topo_path = "./cake-data/topology.yml";
  std::string output, worker;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* name) -> std::string {
      if (i + 1 >= argc) { std::cerr << name << " needs a value\n"; std::exit(2); }
      return argv[++i];
    };
    if (a == "--model-path") model_path = val("--model-path");
    else if (a == "--topology") topo_path = val("--topology");
    else if (a == "--output") output = val("--output");
    else if (a == "--worker") worker = val("--worker");
    else if (a == "-h" || a == "--help") { usage(); return 0; }
    else { std::cerr << "unknown argument " << a << "\n"; usage(); return 2; }
  }
  if (output.empty()) { usage(); return 2; }
  try {
    const Topology topo = Topology::from_path(topo_path, /*text_model=*/true);
    const auto wm = load_weight_map(model_path);
    std::cout << "index has " << wm.size() << " tensors\n";
    std::vector<std::string> selected;
    if (!worker.empty()) selected.push_back(worker);
    else for (const auto& n : topo.nodes) selected.push_back(n.name);
    std::cout << "processing " << selected.size() << " workers\n";
    for (const auto& wname : selected) {
      const TopoNode* node = topo.find(wname);
      if (!node) throw std::runtime_error("can't find worker topology for " + wname);
      std::cout << "processing worker " << wname << " (" << node->host << ") ...\n";
      // shard file -> tensor names owned by this worker
      std::map<std::string, std::vector<std::string>> reduced;
      for (const auto& kv : wm)
        if (node->is_text_model_layer_owner(kv.first)) reduced[kv.second].push_back(kv.first);
      std::vector<std::unique_ptr<SafeTensorsFile>> open;
      std::vector<TensorToWrite> out;
      Json index = Json::object();
      Json wmap = Json::object();
      for (const auto& kv : reduced) {
        std::cout << "loading " << model_path << "/" << kv.first << " ...\n";
        open.push_back(std::make_unique<SafeTensorsFile>(model_path + "/" + kv.first));
        std::cout << "  extracting " << kv.second.size() << " tensors\n";
        for (const auto& tn : kv.second) {
          const TensorView& v = open.back()->tensor(tn);
          out.push_back({v.name, v.dtype, v.shape, v.data, v.nbytes});
          wmap.set(tn, Json::string("reduced.safetensors"));
        }
      }
      index.set("weight_map", std::move(wmap));
      const std::string bundle = output + "/" + wname + "-node";
      const std::string mdir = bundle + "/model";
      mkdirs(mdir);
      std::cout << "compacting " << out.size() << " tensors ...\n";
      {
        std::ofstream f(mdir + "/model.safetensors.index.json");
        f << index.dump(2);
      }
      write_safetensors(mdir + "/reduced.safetensors", out);
      {
        SafeTensorsFile check(mdir + "/reduced.safetensors");  // sanity re-open
        if (check.names().size() != out.size()) throw std::runtime_error("verification failed");
      }
      for (const char* extra : {"config.json", "tokenizer.json", "tokenizer_config.json",
                                "generation_config.json"})
        if (exists(model_path + "/" + extra)) copy_file(model_path + "/" + extra, mdir + "/" + extra);
      Topology single;
      single.nodes.push_back(*node);
      std::ofstream tf(bundle + "/topology.yml");
      tf << single.to_yaml();
      std::cout << "saved " << bundle << "\n";
    }
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << "\n";
    return 1;
  }
  return 0;
}
