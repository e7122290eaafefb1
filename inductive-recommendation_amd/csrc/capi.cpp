// capi.cpp - error reporting and device queries of the igr C ABI.
#include <cstring>
#include <string>

#include "common.h"

namespace igr {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
}  // namespace igr

extern "C" const char *igr_last_error(void) { return igr::g_last_error.c_str(); }

// 1.0.0
extern "C" int igr_version(void) { return 10000; }

extern "C" int igr_device_info(int device, int *n_cu, int *l2_bytes, char *arch, int arch_len) {
    return igr::guarded("igr_device_info", [&]() -> int {
        hipDeviceProp_t p;
        hipError_t e = hipGetDeviceProperties(&p, device);
        if (e != hipSuccess) {
            igr::set_error(std::string("igr_device_info: ") + hipGetErrorString(e));
            return IGR_ERR_HIP;
        }
        if (n_cu) *n_cu = p.multiProcessorCount;
        if (l2_bytes) *l2_bytes = p.l2CacheSize;
        if (arch && arch_len > 0) {
            std::strncpy(arch, p.gcnArchName, (size_t)arch_len - 1);
            arch[arch_len - 1] = 0;
        }
        return IGR_OK;
    });
}
