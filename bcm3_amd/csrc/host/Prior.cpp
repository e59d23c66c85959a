// Prior.cpp -- see Prior.h.
#include "Prior.h"

#include <cmath>
#include <limits>

#include "../../../include/bcm3hip.h"
#include "log.h"

namespace bcm3 {

static const double kInf = std::numeric_limits<double>::infinity();

// UnivariateMarginal::Initialize (UnivariateMarginal.cpp:25-101) for one <variable>
static bool ParseMarginal(const XmlNode& v, Marginal& m)
{
    const std::string dist = v.get("distribution");
    auto f = [&](const char* k) { return v.get_double(k); };
    if (dist == "uniform") {
        const double a = f("lower"), b = f("upper");
        if (b <= a) {
            LOGERROR("Uniform distribution with upper bound less than or equal to lower bound.");
            return false;
        }
        m.kind = BCM3HIP_PRIOR_UNIFORM;
        m.p0 = a;
        m.p1 = b;
    } else if (dist == "normal") {
        const double mu = f("mu"), sigma = f("sigma");
        if (sigma <= 0.0) {
            LOGERROR("Normal distribution with non-positive sigma.");
            return false;
        }
        m.kind = BCM3HIP_PRIOR_NORMAL;
        m.p0 = mu;
        m.p1 = sigma;
    } else if (dist == "exponential") {
        m.kind = BCM3HIP_PRIOR_EXPONENTIAL;
        m.p0 = f("lambda");
        if (m.p0 <= 0.0) {
            LOGERROR("Exponential distribution with non-positive lambda.");
            return false;
        }
    } else if (dist == "gamma") {
        m.kind = BCM3HIP_PRIOR_GAMMA;
        m.p0 = f("k");
        m.p1 = f("theta");
        if (m.p0 <= 0.0 || m.p1 <= 0.0) {
            LOGERROR("Gamma distribution with non-positive k or theta.");
            return false;
        }
    } else if (dist == "beta") {
        m.kind = BCM3HIP_PRIOR_BETA;
        m.p0 = f("a");
        m.p1 = f("b");
        if (m.p0 <= 0.0 || m.p1 <= 0.0) {
            LOGERROR("Beta distribution with non-positive a or b.");
            return false;
        }
    } else if (dist == "half_cauchy") {
        m.kind = BCM3HIP_PRIOR_HALF_CAUCHY;
        m.p0 = f("scale");
        if (m.p0 <= 0.0) {
            LOGERROR("Half-Cauchy distribution with non-positive scale.");
            return false;
        }
    } else if (dist == "beta_prime") {
        m.kind = BCM3HIP_PRIOR_BETA_PRIME;
        m.p0 = f("a");
        m.p1 = f("b");
        m.p2 = f("scale");
    } else if (dist == "exponential_mix") {
        m.kind = BCM3HIP_PRIOR_EXPONENTIAL_MIX;
        m.p0 = f("lambda");
        m.p1 = f("lambda2");
        m.p2 = f("mix");
    } else {
        LOGERROR("Invalid distribution type \"%s\"", dist.c_str());
        return false;
    }
    // GetLowerBound / GetUpperBound (:627-647)
    switch (m.kind) {
    case BCM3HIP_PRIOR_UNIFORM: m.lower = m.p0; m.upper = m.p1; break;
    case BCM3HIP_PRIOR_BETA: m.lower = 0.0; m.upper = 1.0; break;
    case BCM3HIP_PRIOR_EXPONENTIAL:
    case BCM3HIP_PRIOR_GAMMA:
    case BCM3HIP_PRIOR_HALF_CAUCHY:
    case BCM3HIP_PRIOR_BETA_PRIME: m.lower = 0.0; m.upper = kInf; break;
    default: m.lower = -kInf; m.upper = kInf; break;
    }
    // EvaluateMean / EvaluateVariance (:448-540)
    const double p0 = m.p0, p1 = m.p1, p2 = m.p2;
    switch (m.kind) {
    case BCM3HIP_PRIOR_UNIFORM: {
        const double d = p1 - p0;
        m.mean = 0.5 * (p1 + p0);
        m.var = (d * d) / 12.0;
        break;
    }
    case BCM3HIP_PRIOR_NORMAL: m.mean = p0; m.var = p1 * p1; break;
    case BCM3HIP_PRIOR_EXPONENTIAL: m.mean = 1.0 / p0; m.var = 1.0 / (p0 * p0); break;
    case BCM3HIP_PRIOR_GAMMA: m.mean = p0 * p1; m.var = p0 * p1 * p1; break;
    case BCM3HIP_PRIOR_BETA: {
        const double apb = p0 + p1;
        m.mean = p0 / apb;
        m.var = (p0 * p1) / (apb * apb * (apb + 1));
        break;
    }
    case BCM3HIP_PRIOR_HALF_CAUCHY: m.mean = p0; m.var = p0 * p0; break;
    case BCM3HIP_PRIOR_BETA_PRIME:
        m.mean = (p1 > 1.0) ? p2 * p0 / (p1 - 1) : p2;
        m.var = (p1 > 2.0) ? (p2 * p2 * p0 * (p0 + p1 - 1.0) / ((p1 - 2) * (p1 - 1) * (p1 - 1))) : p2 * p2;
        break;
    default:
        m.mean = p2 / p0 + (1.0 - p2) / p1;
        m.var = p2 * p2 / (p0 * p0) + (1.0 - p2) * (1.0 - p2) / (p1 * p1);
        break;
    }
    return true;
}

bool LoadPriorMarginals(const XmlNode& root, std::vector<Marginal>& out)
{
    const XmlNode* node = root.child("prior");
    if (!node) node = root.child("variableset");
    if (!node) {
        LOGERROR("Incorrect prior XML format");
        return false;
    }
    out.clear();
    // multivariate (Dirichlet) groups by id: first variable index and member alphas
    // (PriorIndependence::LoadFromXML, PriorIndependence.cpp:20-115)
    struct Group {
        long first = -1;
        std::vector<double> alpha;
    };
    std::vector<Group> groups;
    std::vector<long> member_group;  // per variable, -1 for univariate
    try {
        for (auto& var : node->children) {
            if (var->name != "variable") continue;
            const bool multivariate = var->get_bool("multivariate", false);
            const long repeat = var->get_long("repeat", 1);
            if (multivariate) {
                if (repeat > 1) {
                    LOGERROR("Multivariate prior with repeat not supported");
                    return false;
                }
                const long id = var->get_long("id", 0);  // missing: the reference throws; 0 is refused below
                if (id <= 0) {
                    LOGERROR("Multivariate distribution IDs should start at 1.");
                    return false;
                }
                const long vix = (long)out.size();
                if (id > (long)groups.size()) groups.resize(id);
                Group& g = groups[id - 1];
                if (g.first < 0) {
                    // the group's first member names its distribution; only dirichlet
                    // (PriorIndependence.cpp:47-51), checked whatever order the ids come in
                    if (var->get("distribution") != "dirichlet") {
                        LOGERROR("Multivariate distribution of unknown type (only dirichlet supported).");
                        return false;
                    }
                    g.first = vix;
                }
                g.alpha.push_back(var->get_double("alpha"));
                if (vix != g.first + (long)g.alpha.size() - 1) {
                    LOGERROR("All variables in a multivariate distribution should follow each other directly");
                    return false;
                }
                Marginal m;
                m.kind = BCM3HIP_PRIOR_DIRICHLET;
                m.p0 = g.alpha.back();
                m.p1 = (double)g.first;
                m.lower = 0.0;  // MultivariateMarginal::GetLowerBound / GetUpperBound (:160-180)
                m.upper = 1.0;
                out.push_back(m);
                member_group.push_back(id - 1);
            } else {
                Marginal m;
                if (!ParseMarginal(*var, m)) return false;
                for (long i = 0; i < repeat; i++) {
                    out.push_back(m);
                    member_group.push_back(-1);
                }
            }
        }
    } catch (XmlError& e) {
        LOGERROR("Error parsing UnivariateMarginal: %s", e.what.c_str());
        return false;
    }
    // MultivariateMarginal::Initialize (:47-64): log normalisation constant; EvaluateMarginalMean /
    // EvaluateMarginalVariance (:120-158) for the proposals' starting moments. lgamma: glibc here,
    // boost::math::lgamma in the reference (parity of this constant unpinned, Boost absent)
    for (size_t gi = 0; gi < groups.size(); gi++) {
        const Group& g = groups[gi];
        if (g.first < 0) {
            LOGERROR("Multivariate distribution id %zu has no variables", gi + 1);
            return false;
        }
        double sum = 0.0, lprod = 0.0;
        for (double a : g.alpha) {
            sum += a;
            lprod += std::lgamma(a);
        }
        const double lnc = std::lgamma(sum) - lprod;
        for (size_t k = 0; k < g.alpha.size(); k++) {
            Marginal& m = out[g.first + k];
            m.p2 = lnc;
            m.mean = g.alpha[k] / sum;
            m.var = g.alpha[k] * (sum - g.alpha[k]) / (sum * sum * (sum + 1.0));
        }
    }
    return true;
}

bool LoadPriorMarginals(const std::string& prior_xml, std::vector<Marginal>& out)
{
    try {
        auto root = xml_load(prior_xml);
        return LoadPriorMarginals(*root, out);
    } catch (XmlError& e) {
        LOGERROR("Error loading prior file: %s", e.what.c_str());
        return false;
    }
}

}  // namespace bcm3
