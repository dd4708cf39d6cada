p='hpgq_engine_tri.h'
s=open(p).read()
a="""    if (NX && !SUB) {   // N | out-of-range << 16 over the lane's valid bytes (as engine_kernel)
      uint32_t nn = 0, oo = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const uint32_t m80 = mk[w] & 0x80808080u;
        if (x_n) nn += (uint32_t)__builtin_popcount(zero_bytes(sw[w] ^ 0x4E4E4E4Eu) & m80);"""
b="""    if (NX && !SUB) {   // N | out-of-range << 16 over the lane's valid bytes (as engine_kernel)
      uint32_t nn = 0, oo = 0;
      // every valid byte exactly A/C/G/T/N (the usual step): N = valid bytes -
      // (C + G) - (A + T), from the codes the step already has (one v_perm and
      // one v_bcnt per word instead of the zero-byte test)
      const bool n_fast = x_n && __ballot(bad != 0u) == 0ull;
      if (n_fast) {
        uint32_t at_n = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) at_n += (uint32_t)__builtin_popcount(__builtin_amdgcn_perm(kATHi, kATLo, cd[w]));
        nn = (uint32_t)min(max((int)(pd.n & 0xFFFFu) - p0, 0), 4 * NW) - gc - at_n;
      }
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const uint32_t m80 = mk[w] & 0x80808080u;
        if (x_n && !n_fast) nn += (uint32_t)__builtin_popcount(zero_bytes(sw[w] ^ 0x4E4E4E4Eu) & m80);"""
assert s.count(a)==1; s=s.replace(a,b); open(p,'w').write(s)
