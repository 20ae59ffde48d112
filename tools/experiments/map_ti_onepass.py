# map TI store: all of a thread's partition-delta quads requested in one round (8 quads: no loop-head wait
# on the previous round's pair stores) instead of two rounds of four
EDITS = [("""    // rate; the pair stores stay 2 bytes per cell)
    constexpr int MQ = MAP_MB / 2;""", """    // rate; the pair stores stay 2 bytes per cell)
    constexpr int MQ = MAP_MB;""")]
