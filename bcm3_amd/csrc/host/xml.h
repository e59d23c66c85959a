// xml.h -- minimal XML reader for BCM3's prior.xml / likelihood.xml (replaces the
// boost::property_tree::read_xml + ptree "<xmlattr>" access used by the reference, e.g.
// src/sampler/VariableSet.cpp:16-69, src/likelihoods/LikelihoodFactory.cpp:31-100).
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace bcm3 {

struct XmlNode {
    std::string name;
    std::map<std::string, std::string> attr;
    std::vector<std::unique_ptr<XmlNode>> children;
    std::string text;

    const XmlNode* child(const std::string& n) const;
    std::vector<const XmlNode*> children_named(const std::string& n) const;
    bool has_attr(const std::string& k) const { return attr.count(k) > 0; }
    // ptree::get<std::string>("<xmlattr>.k") semantics: throws XmlError if missing
    const std::string& get(const std::string& k) const;
    // ptree::get<double>("<xmlattr>.k", default): default when missing OR unparsable (as Boost's
    // get-with-default, cf. width="=0.1" in examples/multimodal_circular_ridge/likelihood.xml)
    double get_double(const std::string& k, double def) const;
    double get_double(const std::string& k) const;  // throws if missing / unparsable
    long get_long(const std::string& k, long def) const;
    bool get_bool(const std::string& k, bool def) const;
};

struct XmlError {
    std::string what;
};

// Parse a document; returns the (virtual) root whose children are the top-level elements.
std::unique_ptr<XmlNode> xml_parse(const std::string& text);
std::unique_ptr<XmlNode> xml_load(const std::string& filename);

}  // namespace bcm3
