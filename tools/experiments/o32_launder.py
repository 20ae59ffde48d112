EDITS = [("""  for (int k = 0; k < nk; k++) {
    const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);
    (void)frame;""", """  for (int k = 0; k < nk; k++) {
    // the thread index laundered per iteration: every per-thread address below is recomputed in the
    // iteration instead of being hoisted out of the loop and held in registers across it
    uint32_t tl = (uint32_t)tid;
    asm volatile("" : "+v"(tl));
    const int tid = (int)tl;
    const uint32_t ta = o32_ta(tl), tb = o32_tb(tl);
    const uint32_t kin = ta + 32u * tb;
    const uint32_t dummy = (uint32_t)(O32_H + (O32_H >> O32_PS)) + (tl & 63u);"""),
]
