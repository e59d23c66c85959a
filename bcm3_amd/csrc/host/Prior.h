// Prior.h -- PriorIndependence over UnivariateMarginal (src/sampler/PriorIndependence.cpp:18-157,
// src/sampler/UnivariateMarginal.cpp:25-101 Initialize, :448-540 moments, :627-647 bounds) as the
// device sampler needs it: per variable the BCM3HIP_PRIOR_* kind and parameters (p0, p1, p2) the
// propose kernels evaluate, the bounds ReflectOnBounds uses, and the marginal mean / variance
// the proposals start from. Density and sampling run on the device (csrc/prior_marginal.h).
#pragma once
#include <string>
#include <vector>

#include "xml.h"

namespace bcm3 {

struct Marginal {
    int kind = 0;  // BCM3HIP_PRIOR_*
    double p0 = 0.0, p1 = 0.0, p2 = 0.0;
    double lower = 0.0, upper = 0.0;  // GetLowerBound / GetUpperBound
    double mean = 0.0, var = 0.0;     // EvaluateMean / EvaluateVariance
};

// <prior><variable name distribution ... [repeat]/>...</prior>, repeat-expanded in order
bool LoadPriorMarginals(const std::string& prior_xml, std::vector<Marginal>& out);
bool LoadPriorMarginals(const XmlNode& root, std::vector<Marginal>& out);

}  // namespace bcm3
