// Test infrastructure (not product code): the few declarations of the reference's src/utils/Utils.h
// that src/sampler/Likelihood.h and a likelihood plugin need, so a plugin written against the
// reference's interface compiles here. Real / VectorReal as src/utils/Typedefs.h:4-5 (Eigen from
// the reference's vendored copy); the Boost types Likelihood::Initialize takes are stand-ins with
// the members a plugin calls (ptree::get, variables_map::operator[]().as<T>()), since Boost is not
// in this image.
#pragma once

#include <cstdio>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include <Eigen/Dense>

namespace bcm3 {
typedef double Real;
typedef Eigen::VectorXd VectorReal;
typedef Eigen::MatrixXd MatrixReal;
}  // namespace bcm3

#define LOG(...) (std::fprintf(stdout, __VA_ARGS__), std::fputc('\n', stdout))
#define LOGERROR(...) (std::fprintf(stderr, __VA_ARGS__), std::fputc('\n', stderr))

namespace boost {
namespace property_tree {
// <bcm_likelihood ...> as boost::property_tree::ptree holds it after read_xml: attribute a at
// "<xmlattr>.a"
class ptree {
public:
    std::map<std::string, std::string> data;
    template <class T>
    T get(const std::string& path) const
    {
        auto it = data.find(path);
        if (it == data.end()) throw std::runtime_error("No such node (" + path + ")");
        return convert<T>(it->second);
    }
    template <class T>
    T get(const std::string& path, const T& def) const
    {
        auto it = data.find(path);
        return it == data.end() ? def : convert<T>(it->second);
    }

private:
    template <class T>
    static T convert(const std::string& s)
    {
        std::istringstream is(s);
        T v{};
        is >> v;
        return v;
    }
};
template <>
inline std::string ptree::convert<std::string>(const std::string& s)
{
    return s;
}
}  // namespace property_tree
namespace program_options {
class variable_value {
public:
    std::string text;
    template <class T>
    T as() const;
};
template <>
inline std::string variable_value::as<std::string>() const
{
    return text;
}
class variables_map {
public:
    std::map<std::string, variable_value> values;
    const variable_value& operator[](const std::string& key) const
    {
        auto it = values.find(key);
        if (it == values.end()) throw std::runtime_error("unrecognised option " + key);
        return it->second;
    }
};
}  // namespace program_options
}  // namespace boost
