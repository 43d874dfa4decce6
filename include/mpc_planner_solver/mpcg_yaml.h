// mpcg_yaml.h — the small YAML subset the solver's generated files use.
//
// The reference reads solver_settings.yaml, parameter_map.yaml and
// model_map.yaml (written by PyYAML's `yaml.dump(..., default_flow_style=False)`,
// solver_generator/util/files.py:110-112) and the planner's settings.yaml
// through yaml-cpp (`loadConfigYaml`, mpc_planner_util/load_yaml.hpp).  yaml-cpp
// is not a dependency here; this reader covers what those files contain:
// block maps, block sequences (also at the parent key's indentation, as PyYAML
// writes them), flow sequences of scalars, quoted / plain scalars, comments.
// The node API is the yaml-cpp subset the solver surface exposes
// (`node["key"][1].as<int>()`, `IsDefined()`, iteration with it->first / it->second).
#pragma once

#include <cstddef>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace mpcg {

class YamlNode {
public:
    enum class Kind { Undefined, Null, Scalar, Sequence, Map };
    using Entry = std::pair<YamlNode, YamlNode>;  // (key scalar, value)
    using const_iterator = std::vector<Entry>::const_iterator;

    YamlNode() = default;
    static YamlNode scalar(std::string s);
    static YamlNode null();
    static YamlNode sequence();
    static YamlNode map();

    Kind kind() const { return kind_; }
    bool IsDefined() const { return kind_ != Kind::Undefined; }
    bool IsNull() const { return kind_ == Kind::Null; }
    bool IsScalar() const { return kind_ == Kind::Scalar; }
    bool IsSequence() const { return kind_ == Kind::Sequence; }
    bool IsMap() const { return kind_ == Kind::Map; }
    std::size_t size() const;

    // Missing keys / indices give an undefined node (yaml-cpp's const access).
    const YamlNode& operator[](const std::string& key) const;
    const YamlNode& operator[](const char* key) const { return (*this)[std::string(key)]; }
    const YamlNode& operator[](std::size_t i) const;
    const YamlNode& operator[](int i) const { return (*this)[static_cast<std::size_t>(i)]; }

    // Map iteration (entries in file order); empty range for other kinds.
    const_iterator begin() const;
    const_iterator end() const;

    template <class T>
    T as() const;

    // Building
    void push_back(YamlNode v);
    void set(const std::string& key, YamlNode v);
    const std::string& text() const { return text_; }

private:
    Kind kind_ = Kind::Undefined;
    std::string text_;
    std::shared_ptr<std::vector<YamlNode>> seq_;
    std::shared_ptr<std::vector<Entry>> map_;
    std::shared_ptr<std::unordered_map<std::string, std::size_t>> index_;
    const std::string& require_scalar(const char* what) const;
};

template <> int YamlNode::as<int>() const;
template <> unsigned int YamlNode::as<unsigned int>() const;
template <> long YamlNode::as<long>() const;
template <> double YamlNode::as<double>() const;
template <> bool YamlNode::as<bool>() const;
template <> std::string YamlNode::as<std::string>() const;

// Parse a document (throws std::runtime_error with the line number on input
// outside the subset).
YamlNode yaml_parse(const std::string& text);
YamlNode yaml_load_file(const std::string& path);

}  // namespace mpcg

// The node type of the Solver's public _config / _parameter_map / _model_map (the reference's are
// YAML::Node, acados_solver_interface.h:175, state.h:29): yaml-cpp's own where it is on the include
// path, so reference code that hands these members to yaml-cpp links unchanged; this reader's
// otherwise (same access API).  -DMPCG_NO_YAML_CPP keeps this reader with yaml-cpp present.
#if __has_include(<yaml-cpp/yaml.h>) && !defined(MPCG_NO_YAML_CPP)
#include <yaml-cpp/yaml.h>
#define MPCG_YAML_CPP 1
namespace MPCPlanner {
using YamlNode = YAML::Node;
inline YamlNode load_yaml_file(const std::string& path) { return YAML::LoadFile(path); }
}  // namespace MPCPlanner
#else
#define MPCG_YAML_CPP 0
namespace MPCPlanner {
using YamlNode = mpcg::YamlNode;
inline YamlNode load_yaml_file(const std::string& path) { return mpcg::yaml_load_file(path); }
}  // namespace MPCPlanner
#endif
