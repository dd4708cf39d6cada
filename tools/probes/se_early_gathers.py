p='hpgq_engine_tri.h'
s=open(p).read()
# load_block: accept pre-issued trim loads (SE)
old='''  auto load_block = [&](const Unit &U, int tb, uint32_t (&len)[NM], uint32_t (&tw)[NM], uint64_t &dm,
                        const int32_t (&ia)[NM], const int32_t (&ie)[NM], bool dma) __attribute__((always_inline)) {'''
new='''  auto load_block = [&](const Unit &U, int tb, uint32_t (&len)[NM], uint32_t (&tw)[NM], uint64_t &dm,
                        const int32_t (&ia)[NM], const int32_t (&ie)[NM], bool dma,
                        const TrimLoads *pre = nullptr) __attribute__((always_inline)) {'''
assert old in s; s=s.replace(old,new)
old='''    } else if (usual) {
#pragma unroll
      for (int m = 0; m < NM; ++m)
        tl[m] = trim_issue(cold, rq[m], live ? bq[m] + ia[m] : (int)0xC0000000, ie[m] - ia[m]);
    }'''
new='''    } else if (usual) {
#pragma unroll
      for (int m = 0; m < NM; ++m)
        tl[m] = trim_issue(cold, rq[m], live ? bq[m] + ia[m] : (int)0xC0000000, ie[m] - ia[m]);
    }
    const bool pre_ok = NM == 1 && EDIT && pre != nullptr && trim_usual(cold);
    if (pre_ok) tl[0] = *pre;'''
assert old in s; s=s.replace(old,new)
old='''        tw[m] = !live ? 0u : usual ? trim_finish(cold, tl[m], e - a) : trim_word(cold, rq[m], bq[m] + a, e - a);'''
new='''        tw[m] = !live ? 0u : (usual || pre_ok) ? trim_finish(cold, tl[m], e - a) : trim_word(cold, rq[m], bq[m] + a, e - a);'''
assert old in s; s=s.replace(old,new)
# describe_next with optional pre
old='''    auto describe_next = [&]() __attribute__((always_inline)) {'''
new='''    TrimLoads pre_tl;   // single-end: the next unit's trim windows, issued a group early
    auto gather_next = [&]() __attribute__((always_inline)) {
      const bool on = lane < nxt.nr;
      const bool live = on && !(ie[0] - ia[0] > dlim);
      pre_tl = trim_issue(cold_all, rq[0], live ? bq[0] + ia[0] : (int)0xC0000000, ie[0] - ia[0]);
    };
    auto describe_next = [&]() __attribute__((always_inline)) {'''
assert old in s; s=s.replace(old,new)
old='''      load_block(nxt, tb ^ 1, lenn, twn, dmn, ia, ie, true);
      nn2 = it.next();'''
new='''      load_block(nxt, tb ^ 1, lenn, twn, dmn, ia, ie, true, (NM == 1 && EDIT && !FOLLOW) ? &pre_tl : nullptr);
      nn2 = it.next();'''
assert old in s; s=s.replace(old,new)
# run_mate: issue gathers at the top of the last pair (before load g+1)
old='''        if (m == NM - 1 && last) issue_dma();   // (the unit's last group pair)
        load_group(m, tb, nt, g + 1, 1);'''
new='''        if (m == NM - 1 && last) issue_dma();   // (the unit's last group pair)
        if (NM == 1 && EDIT && !FOLLOW && last) gather_next();   // (a group before they are finished)
        load_group(m, tb, nt, g + 1, 1);'''
assert old in s; s=s.replace(old,new)
# wholly deferred path: gather before describe
old='''    } else {
      issue_dma();
      if (LATE) describe_next();
      load_group(0, tb ^ 1, nnt, 0, 0);   // a wholly deferred unit: straight to the next'''
new='''    } else {
      issue_dma();
      if (NM == 1 && EDIT && !FOLLOW) gather_next();
      if (LATE) describe_next();
      load_group(0, tb ^ 1, nnt, 0, 0);   // a wholly deferred unit: straight to the next'''
assert old in s; s=s.replace(old,new)
open(p,'w').write(s)
