# chain FEC BB / LDPC passes as one workgroup per FEC block instead of persistent workgroups (no next-block
# prefetch; avoids the loop-head vmcnt(0) that also waits for the previous block's output stores)
EDITS = [("""  void *args[2] = {(void *)&d, (void *)&io};
  return hipLaunchKernel(fn, dim3(fec_grid(io.nblocks, per_cu)), dim3(FEC_THREADS), args, lds, s);""",
          """  void *args[2] = {(void *)&d, (void *)&io};
  const bool np = kind == CARVE_LDPC;
  return hipLaunchKernel(fn, dim3(np ? io.nblocks : fec_grid(io.nblocks, per_cu)), dim3(FEC_THREADS), args, lds, s);""")]
