#include "topology.h"

#include <fstream>
#include <regex>
#include <sstream>
#include <stdexcept>

namespace cake {

bool TopoNode::is_text_model_layer_owner(const std::string& full_name) const {
  for (const auto& prefix : layers) {
    const std::string p = prefix + ".";
    if (full_name.compare(0, p.size(), p) == 0) return true;
  }
  return false;
}

std::vector<std::string> expand_layer_range(const std::string& spec) {
  static const std::regex re(R"(^(.+[^\d])(\d+)-(\d+)$)");
  std::smatch m;
  if (!std::regex_match(spec, m, re)) return {spec};
  const std::string base = m[1];
  const long start = std::stol(m[2]), stop = std::stol(m[3]);
  if (stop <= start)
    throw std::runtime_error("invalid range expression " + spec + ", end must be > start");
  std::vector<std::string> out;
  for (long n = start; n <= stop; ++n) out.push_back(base + std::to_string(n));
  return out;
}

namespace {

struct Line {
  int indent;
  std::string text;  // comment-stripped, right-trimmed, indentation removed
  int lineno;
};

std::string rtrim(const std::string& s) {
  size_t e = s.find_last_not_of(" \t\r");
  return e == std::string::npos ? "" : s.substr(0, e + 1);
}

std::string trim(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r");
  if (b == std::string::npos) return "";
  return rtrim(s.substr(b));
}

std::string strip_comment(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (c == '#' && !sq && !dq && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t'))
      return s.substr(0, i);
  }
  return s;
}

std::string scalar(const std::string& raw) {
  std::string s = trim(raw);
  if (s.size() >= 2 && ((s.front() == '\'' && s.back() == '\'') ||
                        (s.front() == '"' && s.back() == '"'))) {
    std::string in = s.substr(1, s.size() - 2);
    if (s.front() == '\'') {  // '' -> '
      std::string o;
      for (size_t i = 0; i < in.size(); ++i) {
        o += in[i];
        if (in[i] == '\'' && i + 1 < in.size() && in[i + 1] == '\'') ++i;
      }
      return o;
    }
    std::string o;  // minimal double-quoted escapes
    for (size_t i = 0; i < in.size(); ++i) {
      if (in[i] == '\\' && i + 1 < in.size()) {
        char e = in[++i];
        o += e == 'n' ? '\n' : e == 't' ? '\t' : e;
      } else {
        o += in[i];
      }
    }
    return o;
  }
  if (s == "~" || s == "null") return "";
  return s;
}

std::vector<std::string> flow_list(const std::string& s, int lineno) {
  std::string in = trim(s);
  if (in.size() < 2 || in.front() != '[' || in.back() != ']')
    throw std::runtime_error("line " + std::to_string(lineno) + ": expected [ ... ]");
  in = in.substr(1, in.size() - 2);
  std::vector<std::string> out;
  std::string cur;
  bool sq = false, dq = false;
  for (char c : in) {
    if (c == '\'' && !dq) sq = !sq;
    if (c == '"' && !sq) dq = !dq;
    if (c == ',' && !sq && !dq) {
      if (!trim(cur).empty()) out.push_back(scalar(cur));
      cur.clear();
    } else {
      cur += c;
    }
  }
  if (!trim(cur).empty()) out.push_back(scalar(cur));
  return out;
}

// split "key: value" at the first ':' outside quotes followed by space/end
bool split_kv(const std::string& t, std::string& k, std::string& v) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < t.size(); ++i) {
    char c = t[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (c == ':' && !sq && !dq && (i + 1 == t.size() || t[i + 1] == ' ' || t[i + 1] == '\t')) {
      k = scalar(t.substr(0, i));
      v = trim(t.substr(i + 1));
      return true;
    }
  }
  return false;
}

}  // namespace

Topology Topology::parse(const std::string& yaml, bool text_model) {
  std::vector<Line> lines;
  {
    std::istringstream in(yaml);
    std::string raw;
    int n = 0;
    while (std::getline(in, raw)) {
      ++n;
      std::string s = rtrim(strip_comment(raw));
      if (trim(s).empty() || trim(s) == "---") continue;
      size_t ind = s.find_first_not_of(' ');
      if (s.find('\t') != std::string::npos && s.find('\t') < ind)
        throw std::runtime_error("line " + std::to_string(n) + ": tabs are not valid indentation");
      lines.push_back({(int)ind, s.substr(ind), n});
    }
  }
  Topology topo;
  if (lines.size() == 1 && (lines[0].text == "{}" || lines[0].text == "null")) return topo;
  size_t i = 0;
  while (i < lines.size()) {
    const Line& L = lines[i];
    if (L.indent != 0)
      throw std::runtime_error("line " + std::to_string(L.lineno) + ": expected a worker name");
    std::string name, rest;
    if (!split_kv(L.text, name, rest))
      throw std::runtime_error("line " + std::to_string(L.lineno) + ": expected 'name:'");
    TopoNode node;
    node.name = name;
    bool have_host = false;
    ++i;
    if (!rest.empty() && rest != "{}")
      throw std::runtime_error("line " + std::to_string(L.lineno) + ": inline worker mapping not supported");
    while (i < lines.size() && lines[i].indent > 0) {
      const Line& F = lines[i];
      std::string key, val;
      if (!split_kv(F.text, key, val))
        throw std::runtime_error("line " + std::to_string(F.lineno) + ": expected 'key: value'");
      const int key_indent = F.indent;
      ++i;
      if (key == "layers") {
        if (!val.empty()) {
          node.layers = flow_list(val, F.lineno);
        } else {
          while (i < lines.size() && lines[i].indent >= key_indent &&
                 lines[i].text.rfind("-", 0) == 0) {
            std::string item = lines[i].text.substr(1);
            node.layers.push_back(scalar(item));
            ++i;
          }
        }
      } else {
        // skip any nested block of an unknown key
        if (val.empty())
          while (i < lines.size() && lines[i].indent > key_indent) ++i;
        if (key == "host") { node.host = scalar(val); have_host = true; }
        else if (key == "description") { node.description = scalar(val); node.has_description = true; }
      }
    }
    if (!have_host) throw std::runtime_error("worker '" + name + "' has no host");
    if (text_model) {
      std::vector<std::string> expanded;
      for (const auto& l : node.layers)
        for (auto& e : expand_layer_range(l)) expanded.push_back(std::move(e));
      node.layers = std::move(expanded);
    }
    topo.nodes.push_back(std::move(node));
  }
  return topo;
}

Topology Topology::from_path(const std::string& path, bool text_model) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("can't read " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return parse(ss.str(), text_model);
}

const TopoNode* Topology::node_for_layer(const std::string& layer) const {
  for (const auto& n : nodes)
    for (const auto& l : n.layers)
      if (l == layer) return &n;
  return nullptr;
}

const TopoNode* Topology::find(const std::string& name) const {
  for (const auto& n : nodes)
    if (n.name == name) return &n;
  return nullptr;
}

std::string Topology::to_yaml() const {
  std::ostringstream o;
  for (const auto& n : nodes) {
    o << n.name << ":\n  host: '" << n.host << "'\n";
    if (n.has_description) o << "  description: '" << n.description << "'\n";
    o << "  layers:\n";
    for (const auto& l : n.layers) o << "  - " << l << "\n";
  }
  return o.str();
}

}  // namespace cake
