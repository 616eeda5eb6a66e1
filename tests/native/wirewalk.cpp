// CPU driver for the host part of drb_ingest_wire (drb_wirehost.hpp), built
// by tests/test_wirehost.py with -fsanitize=address,undefined.  Reads one
// stream file and prints what the walk made of it, one line per frame:
//   frame <off> <size> <method> <crc_ok> <scan_ok> <did> <bv> <wide> <steps...>
// then "walked <bytes> bad <0|1>".  The frames are scanned by several
// threads at once, as drb_ingest_wire does.  Test infrastructure only.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <thread>

#include "../../dragonboat_amd/csrc/drb_wirehost.hpp"

int main(int argc, char **argv) {
  if (argc != 2) return 2;
  FILE *fp = fopen(argv[1], "rb");
  if (!fp) return 2;
  std::vector<uint8_t> buf;
  uint8_t tmp[65536];
  size_t n;
  while ((n = fread(tmp, 1, sizeof(tmp), fp)) > 0)
    buf.insert(buf.end(), tmp, tmp + n);
  fclose(fp);
  // an exact-size heap copy: a read past the stream's end is an ASan error
  uint8_t *stream = buf.empty() ? nullptr : (uint8_t *)malloc(buf.size());
  if (stream) memcpy(stream, buf.data(), buf.size());
  const size_t len = buf.size();
  wirehost::crc_init();
  std::vector<wirehost::Frame> fr;
  bool bad = false;
  // twice: the second call reuses the frame vectors (a warm call)
  size_t walked = 0;
  for (int pass = 0; pass < 2; ++pass) {
    walked = wirehost::walk_frames(stream, len, fr, &bad);
    const size_t nt = std::min<size_t>(4, fr.size());
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt; ++t)
      th.emplace_back([&, t]() {
        for (size_t f = t; f < fr.size(); f += nt)
          if (fr[f].method == 100) wirehost::scan_batch(stream, fr[f]);
      });
    for (auto &x : th) x.join();
  }
  for (const auto &f : fr) {
    // the payload CRC as the GPU computes it: 16 KB chunks' raw CRCs,
    // folded and conditioned on the host
    std::vector<uint32_t> raw, cl;
    for (uint64_t o = 0; o < f.size; o += 16384) {
      const uint32_t l = (uint32_t)std::min<uint64_t>(16384, f.size - o);
      raw.push_back(wirehost::crc_raw(stream + f.off + o, l));
      cl.push_back(l);
    }
    const uint32_t c =
        wirehost::fold_frame_crc(raw.data(), cl.data(), raw.size(), f.size);
    const bool crc_ok = c == f.pcrc && c == wirehost::crc32_small(
                                               stream + f.off, f.size);
    std::vector<uint16_t> s16(f.step.size() + 1);
    const bool narrow = wirehost::pack_steps16(f, s16.data());
    printf("frame %llu %llu %u %d %d %llu %llu %d", (unsigned long long)f.off,
           (unsigned long long)f.size, f.method, crc_ok ? 1 : 0,
           f.scan_ok ? 1 : 0, (unsigned long long)f.did,
           (unsigned long long)f.bv, narrow ? 0 : 1);
    for (size_t k = 0; k < f.step.size(); ++k) {
      if (narrow && s16[k] != f.step[k]) return 3;
      printf(" %u", f.step[k]);
    }
    printf("\n");
  }
  printf("walked %zu bad %d\n", walked, bad ? 1 : 0);
  free(stream);
  return 0;
}
