// capi_output.cpp -- include/bcm3.h's bcm3_samples_* entry points on SampleFileWriter.
#include <string>
#include <vector>

#include "../../../include/bcm3.h"
#include "NetCDFClassic.h"
#include "log.h"

struct bcm3_samples {
    bcm3::SampleFileWriter w;
    int32_t d = 0;
};

extern "C" {

int bcm3_samples_open(const char* filename, int64_t num_samples, int32_t d, const char* const* names,
                      const int32_t* transforms, int32_t num_temperatures, const double* temperatures, int32_t first,
                      int32_t own, bcm3_samples** out)
{
    if (!filename || !names || !transforms || !temperatures || !out || d < 1 || num_temperatures < 1 || first < 0 ||
        own < 0)
        return -1;
    *out = nullptr;
    std::vector<std::string> nm(names, names + d);
    std::vector<int32_t> tr(transforms, transforms + d);
    std::vector<double> temps(temperatures, temperatures + num_temperatures);
    auto h = new bcm3_samples;
    h->d = d;
    if (!h->w.Initialize(filename, (size_t)num_samples, nm, tr, temps, (size_t)first, (size_t)own)) {
        delete h;
        return -2;
    }
    *out = h;
    return 0;
}

int bcm3_samples_write(bcm3_samples* h, int64_t sample_ix, int32_t t0, int32_t nt, const double* values,
                       const double* lprior, const double* llh, const double* weight)
{
    if (!h || !values || !lprior || !llh || !weight || sample_ix < 0 || t0 < 0 || nt < 0) return -1;
    return h->w.Write((size_t)sample_ix, (size_t)t0, (size_t)nt, values, lprior, llh, weight) ? 0 : -2;
}

int bcm3_samples_sync(bcm3_samples* h) { return (h && h->w.Sync()) ? 0 : -2; }

void bcm3_samples_close(bcm3_samples* h) { delete h; }
}
