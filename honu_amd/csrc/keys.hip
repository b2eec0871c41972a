// keys.hip — Object.Key() over a batch (object.go:57-64 -> keys.New,
// keys/keys.go:42-51): the 29-byte key column from decoded rows.
#include "kernels.h"

namespace honu {

// ------------------------------------------------------------------------
// keys: Object.Key() -> keys.New(ObjectID, &Version.Scalar) (keys.go:42-51)
// ------------------------------------------------------------------------
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_keys(const honu_meta *__restrict__ meta,
                                                            const honu_record_info *__restrict__ info,
                                                            uint64_t n, uint8_t *__restrict__ keys,
                                                            int32_t *__restrict__ key_status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const honu_meta &m = meta[i];
    int32_t st = info[i].meta_status;
    if (st == HONU_OK && !(m.present & HONU_HAS_VERSION)) st = HONU_ERR_PANIC;  // metadata.go:54
    uint8_t *k = keys + HONU_KEY_LEN * i;
    if (st == HONU_OK) {
        k[0] = 0x01;  // keyVersion keys.go:18
        for (int j = 0; j < 16; j++) k[1 + j] = m.object_id[j];
        for (int j = 0; j < 8; j++) k[17 + j] = (uint8_t)(m.vid >> (56 - 8 * j));  // BE64(VID)
        for (int j = 0; j < 4; j++) k[25 + j] = (uint8_t)(m.pid >> (24 - 8 * j));  // BE32(PID)
    } else {
        for (int j = 0; j < HONU_KEY_LEN; j++) k[j] = 0;
    }
    if (key_status) key_status[i] = st;
}

hipError_t launch_decode_keys(const LaunchGeom &g, const honu_meta *meta,
                              const honu_record_info *info, uint64_t n, uint8_t *keys,
                              int32_t *key_status, hipStream_t s) {
    (void)g;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, meta,
                       info, n, keys, key_status);
    return hipGetLastError();
}

}  // namespace honu
