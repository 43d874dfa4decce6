// TEST INFRASTRUCTURE ONLY (tests/test_cpp_yaml_api.py): yaml-cpp is not installed in this image, so
// this header stands in for <yaml-cpp/yaml.h> with the part of YAML::Node's API the drop-in Solver and
// reference-style callers use (operator[], as<T>(), IsDefined(), size(), iteration through
// YAML::const_iterator with it->first / it->second, YAML::LoadFile), implemented over the drop-in's
// own reader.  It proves that the drop-in's yaml-cpp branch (mpcg_yaml.h: MPCPlanner::YamlNode =
// YAML::Node) compiles and runs against that API; it is never part of a product build.
#pragma once
#include <string>
#include <utility>

#include "mpc_planner_solver/mpcg_yaml.h"

namespace YAML {
class const_iterator;
class Node {
public:
    Node() = default;
    Node(mpcg::YamlNode n) : n_(std::move(n)) {}
    Node operator[](const std::string& k) const { return Node(n_[k]); }
    Node operator[](const char* k) const { return Node(n_[k]); }
    Node operator[](int i) const { return Node(n_[i]); }
    Node operator[](std::size_t i) const { return Node(n_[i]); }
    bool IsDefined() const { return n_.IsDefined(); }
    bool IsMap() const { return n_.IsMap(); }
    bool IsSequence() const { return n_.IsSequence(); }
    std::size_t size() const { return n_.size(); }
    template <class T>
    T as() const { return n_.as<T>(); }
    const_iterator begin() const;
    const_iterator end() const;

private:
    mpcg::YamlNode n_;
};
struct iterator_value {
    Node first, second;
};
class const_iterator {
public:
    explicit const_iterator(mpcg::YamlNode::const_iterator it) : it_(it) {}
    const iterator_value* operator->() const { v_ = iterator_value{Node(it_->first), Node(it_->second)}; return &v_; }
    const iterator_value& operator*() const { return *operator->(); }
    const_iterator& operator++() { ++it_; return *this; }
    bool operator!=(const const_iterator& o) const { return it_ != o.it_; }
    bool operator==(const const_iterator& o) const { return it_ == o.it_; }

private:
    mpcg::YamlNode::const_iterator it_;
    mutable iterator_value v_;
};
inline const_iterator Node::begin() const { return const_iterator(n_.begin()); }
inline const_iterator Node::end() const { return const_iterator(n_.end()); }
inline Node LoadFile(const std::string& path) { return Node(mpcg::yaml_load_file(path)); }
}  // namespace YAML
