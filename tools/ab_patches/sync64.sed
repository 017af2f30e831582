s/^__global__ __launch_bounds__(64 \* SYNC_WAVES) void k_etsi_sync(/__global__ __launch_bounds__(64 * SYNC_WAVES) __attribute__((amdgpu_waves_per_eu(8))) void k_etsi_sync(/
