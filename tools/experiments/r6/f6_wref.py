# experiment: the build works on the TS window's slot by reference (no by-value copy)
EDITS = [('    auto build = [&](int q, TsWin w, uint32_t *pd) {', "    auto build = [&](int q, TsWin &w, uint32_t *pd) {   // w: the window's slot, fixed up in place on an edge"), ('    auto chunk = [&](int q, const TsWin &wn, TsWin &wl) {', '    auto chunk = [&](int q, TsWin &wn, TsWin &wl) {')]
