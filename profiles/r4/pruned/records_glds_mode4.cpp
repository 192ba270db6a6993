  if (mode == 4) {  // LDS-DMA staged gather (A/B; whole 16-byte input chunks only)
    if (aligned && rb >= 16 && rb <= 244 && ((nin * (u64)rb) & 15) == 0) {
      switch ((rb + 27) / 16) {
        case 2: launch_gather_glds<2>(in, nin, perm, n, rb, out, s); break;
        case 3: launch_gather_glds<3>(in, nin, perm, n, rb, out, s); break;
        case 4: launch_gather_glds<4>(in, nin, perm, n, rb, out, s); break;
        case 5: launch_gather_glds<5>(in, nin, perm, n, rb, out, s); break;
        case 6: launch_gather_glds<6>(in, nin, perm, n, rb, out, s); break;
        case 7: launch_gather_glds<7>(in, nin, perm, n, rb, out, s); break;
        case 8: launch_gather_glds<8>(in, nin, perm, n, rb, out, s); break;
        case 9: launch_gather_glds<9>(in, nin, perm, n, rb, out, s); break;
        case 10: launch_gather_glds<10>(in, nin, perm, n, rb, out, s); break;
        case 11: launch_gather_glds<11>(in, nin, perm, n, rb, out, s); break;
        case 12: launch_gather_glds<12>(in, nin, perm, n, rb, out, s); break;
        case 13: launch_gather_glds<13>(in, nin, perm, n, rb, out, s); break;
        case 14: launch_gather_glds<14>(in, nin, perm, n, rb, out, s); break;
        case 15: launch_gather_glds<15>(in, nin, perm, n, rb, out, s); break;
        default: launch_gather_glds<16>(in, nin, perm, n, rb, out, s); break;
      }
      return (int)hipGetLastError();
    }
    mode = 0;
  }
