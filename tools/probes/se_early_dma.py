p='hpgq_engine_tri.h'
s=open(p).read()
a='constexpr bool TDMA = EDIT && !FOLLOW && NM == 2 && XM == 0;'
assert a in s; s=s.replace(a,'constexpr bool TDMA = EDIT && !FOLLOW && XM == 0;')
old='''      for (int g = 0; g < ngroups; g += 2) {
        const bool last = g + 2 >= ngroups;
        if (m == NM - 1 && last) issue_dma();   // (the unit's last group pair)
        load_group(m, tb, nt, g + 1, 1);
        process_group(g, 0);
        if (NM == 1 && LATE) {
          // edit: ONE load site for slot 0, this unit's next group or the next
          // unit's first, behind the next unit's prologue (round 5: C4 811 ->
          // 806 us; C2, whose else-branch is a plain load, ran 1.5 % slower
          // this way and keeps the if / else)
          if (last) describe_next();
          load_group(0, last ? tb ^ 1 : tb, last ? nnt : nt, last ? 0 : g + 2, 0);
        } else if (!last) {'''
new='''      // single-end TDMA: the DMA goes out a group pair before the prologue
      // (after the second-to-last pair's second group's loads), with three
      // phantom loads (out of range: no traffic) issued after that pair's
      // first group's loads: hipcc's next wait (for that group) then counts
      // three loads younger than it really has, the phantoms absorb the
      // difference instead of the DMA (vmcnt is in order), and the DMA is
      // first drained a whole group later
      const bool early = TDMA && NM == 1 && tdma && ngroups >= 4;
      for (int g = 0; g < ngroups; g += 2) {
        const bool last = g + 2 >= ngroups;
        const bool prev = early && g + 4 >= ngroups && !last;
        if (m == NM - 1 && last && !early) issue_dma();   // (the unit's last group pair)
        load_group(m, tb, nt, g + 1, 1);
        if (prev) {
          ph0 = __builtin_amdgcn_raw_buffer_load_b32(rq[0], 0x80000000u, 0, 0);
          ph1 = __builtin_amdgcn_raw_buffer_load_b32(rq[0], 0x80000004u, 0, 0);
          ph2 = __builtin_amdgcn_raw_buffer_load_b32(rq[0], 0x80000008u, 0, 0);
        }
        process_group(g, 0);
        if (NM == 1 && LATE) {
          // edit: ONE load site for slot 0, this unit's next group or the next
          // unit's first, behind the next unit's prologue (round 5: C4 811 ->
          // 806 us; C2, whose else-branch is a plain load, ran 1.5 % slower
          // this way and keeps the if / else)
          if (last) {
            describe_next();
            if (early) asm volatile("" ::"v"(ph0), "v"(ph1), "v"(ph2));
          }
          load_group(0, last ? tb ^ 1 : tb, last ? nnt : nt, last ? 0 : g + 2, 0);
          if (prev) issue_dma();
        } else if (!last) {'''
assert old in s; s=s.replace(old,new)
# phantom registers declared before the unit loop
old='''  constexpr uint64_t not_seg_first = not_seg_first_mask<G>();   // lanes j with j % kSegs != 0'''
new='''  uint32_t ph0 = 0, ph1 = 0, ph2 = 0;   // single-end TDMA's phantom loads (see run_mate)
  constexpr uint64_t not_seg_first = not_seg_first_mask<G>();   // lanes j with j % kSegs != 0'''
assert old in s; s=s.replace(old,new)
open(p,'w').write(s)
p='hpgq_engine.hip'
s=open(p).read()
a='nm == 2 && xm == 0'
assert a in s; s=s.replace(a,'xm == 0')
open(p,'w').write(s)
