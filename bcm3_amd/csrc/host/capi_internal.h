// capi_internal.h -- the handle behind include/bcm3.h's bcm3_likelihood, shared by the C-ABI files.
#pragma once
#include <memory>

#include "Likelihood.h"

struct bcm3_likelihood {
    std::shared_ptr<bcm3::VariableSet> varset;
    std::shared_ptr<bcm3::Likelihood> ll;
};
