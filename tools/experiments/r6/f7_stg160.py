# experiment: staging row stride 160 B
EDITS = [('constexpr int BBCH_STG_STRIDE = 144;', 'constexpr int BBCH_STG_STRIDE = 160;')]
