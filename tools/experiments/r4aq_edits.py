# 32K OFDM workgroups frame-fast in plain dispatch order (no XCD-major remap): the XCDs' concurrent
# workgroups all hold the same symbol of interleaved frames
EDITS = [(
    """  const int u = xcd_major(blockIdx.x, gridDim.x);
  const int j = u / io.nframes;                   // symbol
  const int f = u - j * io.nframes;               // frame within launch
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);   // stream-major batch
  const float2 *data = io.data;
  const uint32_t cbase""",
    """  const int u = blockIdx.x;
  const int j = u / io.nframes;                   // symbol
  const int f = u - j * io.nframes;               // frame within launch
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);   // stream-major batch
  const float2 *data = io.data;
  const uint32_t cbase""")]
