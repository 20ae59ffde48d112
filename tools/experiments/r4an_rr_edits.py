# (r4an second variant: without the XCD-major order, so the XCDs share the same few frames)
# 32K OFDM workgroups symbol-fast: consecutive logical workgroups take consecutive symbols of one frame
# (each XCD writes a contiguous run of frames' IQ) instead of one symbol of consecutive frames
EDITS = [(
    """  const int u = xcd_major(blockIdx.x, gridDim.x);
  const int j = u / io.nframes;                   // symbol
  const int f = u - j * io.nframes;               // frame within launch
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);   // stream-major batch
  const float2 *data = io.data;
  const uint32_t cbase""",
    """  const int u = blockIdx.x;
  const int f = u / d.Nsym;                       // frame within launch
  const int j = u - f * d.Nsym;                   // symbol
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);   // stream-major batch
  const float2 *data = io.data;
  const uint32_t cbase""")]
