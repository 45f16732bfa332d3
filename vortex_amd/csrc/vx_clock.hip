// vx_clock.hip — shader-clock stamps around a stretch of GPU work (bench
// measurement, not the hashing path).
//
// The config-2 kernel is bound by VALU issue, so its rate is
// set by the shader clock the chip holds while it runs.  bench.py brackets
// its timed steps with two launches of this kernel on the same stream: each
// workgroup's first lane records the shader cycle counter (s_memtime), the
// constant-rate real-time counter (s_memrealtime, 100 MHz on MI355X:
// hipDeviceAttributeWallClockRate) and the XCC it ran on.  Per XCC,
//   clock = (cycles_after - cycles_before) / (rt_after - rt_before) * rt_rate
// is the mean shader clock over the bracketed work.  The stamps are three
// vector stores per workgroup; the kernel reads no memory.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vx_tuning.h"

namespace {

// s_getreg_b32 HW_REG_XCC_ID (hardware register 20 on gfx940/gfx950), bits [3:0]:
// size - 1 = 3 at bit 11, offset 0 at bit 6, register id 20.
constexpr int kXccIdReg = (3 << 11) | (0 << 6) | 20;

__global__ __launch_bounds__(64) void clock_stamp_kernel(uint64_t* __restrict__ out) {
    if (threadIdx.x != 0) return;
    const uint64_t cycles = __builtin_amdgcn_s_memtime();
    const uint64_t rt = __builtin_amdgcn_s_memrealtime();
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(kXccIdReg) & 15u;
    uint64_t* o = out + 3ull * blockIdx.x;
    o[0] = cycles;
    o[1] = rt;
    o[2] = xcc;
}

}  // namespace

extern "C" int vx_tuning_clock_stamp(void* d_out, uint32_t blocks, void* stream) {
    if (!d_out || blocks == 0 || blocks > 65536) return -22;  // VX_EINVAL
    hipLaunchKernelGGL(clock_stamp_kernel, dim3(blocks), dim3(64), 0, static_cast<hipStream_t>(stream),
                       static_cast<uint64_t*>(d_out));
    return hipGetLastError() == hipSuccess ? 0 : -5;  // VX_EDEVICE
}

// Which physical GPU an ordinal is (bench.py's per-rank identity at N > 1):
// its PCI bus id ("dddd:bb:dd.f") and 16-byte UUID.
extern "C" int vx_tuning_device_identity(int device, char* bus_id, size_t len, char* uuid16) {
    if (!bus_id || len < 16 || !uuid16) return -22;
    if (hipDeviceGetPCIBusId(bus_id, (int)len, device) != hipSuccess) return -5;
    hipUUID u;
    if (hipDeviceGetUuid(&u, device) != hipSuccess) return -5;
    for (int i = 0; i < 16; ++i) uuid16[i] = u.bytes[i];
    return 0;
}

extern "C" int vx_tuning_wall_clock_khz(int device) {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess) return -5;
    return khz;
}
