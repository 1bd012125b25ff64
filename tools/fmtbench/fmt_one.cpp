// fmt_one.cpp - one formatter thread over a resident batch (tools/fmtbench/prep.py
// output in /tmp/fbd), with and without frame header lines; min of 12 runs
// is the number.  Development tool.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "netsniff_dissect.h"
static std::vector<char> rd(const std::string &p) { FILE *f = fopen(p.c_str(), "rb"); fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET); std::vector<char> v(n); if (fread(v.data(), 1, n, f) != (size_t)n) exit(1); fclose(f); return v; }
int main(int argc, char **argv) {
	std::string d = argc > 1 ? argv[1] : "/tmp/fbd";
	auto fr = rd(d + "/frames.bin"), de = rd(d + "/desc.bin"), cr = rd(d + "/crec.bin"), po = rd(d + "/pool.bin"), fh = rd(d + "/fh.bin");
	const uint32_t n = 262144;
	std::vector<char> out((size_t)n * 700);
	for (int rep = 0; rep < 12; rep++)
	for (int withfh = 0; withfh < 2; withfh++) {
		auto t0 = std::chrono::steady_clock::now();
		long r = nsd_format_range_compact_fh((const uint8_t *)fr.data(), (const nsd_desc_t *)de.data(), nullptr,
			withfh ? (const nsd_frame_hdr_t *)fh.data() : nullptr, 1, 0, n, 1, 0, (const nsd_crec *)cr.data(),
			(const uint32_t *)po.data(), out.data(), out.size(), nullptr, nullptr);
		double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
		printf("fh=%d %.1f ns/pkt (%ld B)\n", withfh, dt / n * 1e9, r);
	}
	return 0;
}
