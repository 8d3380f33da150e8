// swimsim_kernels.h — kernel entry points of the engine (defined in swimsim_kernels.hip)
#pragma once
#include "swimsim_device.h"

namespace swimdev {
// maxn bounds the row count on the device
void launch_checksum(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t maxn, hipStream_t s);
void launch_checksum_dump(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t *dbg, uint32_t cap,
                          hipStream_t s);
void launch_checksum_mode(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t maxn, int mode,
                          hipStream_t s);
}
