# experiment: ldpc_map_kernel at 6 workgroups per CU (launch bounds; more VGPRs)
EDITS = [('__global__ __launch_bounds__(FEC_THREADS, FEC_PASS_WG_PER_CU) void ldpc_map_kernel(FecDev fd, FecIO fio, MapDev md,', '__global__ __launch_bounds__(FEC_THREADS, 6) void ldpc_map_kernel(FecDev fd, FecIO fio, MapDev md,')]
