// Forced splits (`forcedsplits_filename`): the JSON tree {"feature": f, "threshold": t,
// "left": {...}, "right": {...}} and its breadth-first flattening for the device learner.
// Reference: serial_tree_learner.cpp:624-738 (ForceSplits, BFS over the JSON).
#pragma once

#include <cctype>
#include <cstdlib>
#include <memory>
#include <queue>
#include <string>
#include <vector>

namespace lgap {

struct ForcedNode {
  int feature = -1;
  double threshold = 0.0;
  std::unique_ptr<ForcedNode> left, right;
};
inline std::unique_ptr<ForcedNode> ParseForced(const std::string& s, size_t* pos) {
  auto skip = [&] { while (*pos < s.size() && std::isspace(static_cast<unsigned char>(s[*pos]))) ++*pos; };
  skip();
  if (*pos >= s.size() || s[*pos] != '{') return nullptr;
  ++*pos;
  auto node = std::make_unique<ForcedNode>();
  while (*pos < s.size()) {
    skip();
    if (s[*pos] == '}') {
      ++*pos;
      break;
    }
    if (s[*pos] == ',') {
      ++*pos;
      continue;
    }
    size_t q1 = s.find('"', *pos), q2 = s.find('"', q1 + 1);
    std::string key = s.substr(q1 + 1, q2 - q1 - 1);
    *pos = s.find(':', q2) + 1;
    skip();
    if (key == "left" || key == "right") {
      auto child = ParseForced(s, pos);
      (key == "left" ? node->left : node->right) = std::move(child);
    } else {
      char* e;
      double v = std::strtod(s.c_str() + *pos, &e);
      *pos = e - s.c_str();
      if (key == "feature") node->feature = static_cast<int>(v);
      else if (key == "threshold") node->threshold = v;
    }
  }
  return node;
}

// One forced split in the order the host learner applies them (ForceSplits: a queue, popped
// front first, children pushed left then right after a split). `valid(feature)` drops nodes
// the host skips (unknown / unused / non-numerical features) together with their subtrees,
// exactly as the host's `continue` never pushes their children. left / right: indices of the
// children in the flattened list, -1 for none.
struct FlatForced {
  int feature;       // raw feature index
  double threshold;  // raw threshold (the caller maps it to a bin)
  int left, right;
};

template <typename Valid>
std::vector<FlatForced> FlattenForced(const ForcedNode* root, Valid valid) {
  std::vector<FlatForced> out;
  if (root == nullptr) return out;
  std::queue<std::pair<const ForcedNode*, std::pair<int, int>>> q;  // node, (parent index, side)
  q.push({root, {-1, 0}});
  while (!q.empty()) {
    auto [n, link] = q.front();
    q.pop();
    if (!valid(n->feature)) continue;
    const int me = static_cast<int>(out.size());
    out.push_back({n->feature, n->threshold, -1, -1});
    if (link.first >= 0) (link.second == 0 ? out[link.first].left : out[link.first].right) = me;
    if (n->left) q.push({n->left.get(), {me, 0}});
    if (n->right) q.push({n->right.get(), {me, 1}});
  }
  return out;
}

}  // namespace lgap
