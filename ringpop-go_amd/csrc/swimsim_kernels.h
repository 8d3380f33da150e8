// swimsim_kernels.h — kernel entry points of the engine (defined in swimsim_kernels.hip)
#pragma once
#include "swimsim_device.h"

namespace swimdev {
// maxn bounds the row count on the device; nrows is the count when the host knows it (else ~0u): it
// picks the latency (few rows) or the throughput variant
void launch_checksum(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t maxn, uint32_t nrows,
                     hipStream_t s);
#ifdef SWIMSIM_DIAG   // diagnostics library only (tools/diag)
void launch_checksum_dump(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t *dbg, uint32_t cap,
                          hipStream_t s);
void launch_checksum_mode(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t maxn, int mode,
                          hipStream_t s);
#endif
}
