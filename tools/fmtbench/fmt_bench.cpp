// fmt_bench.cpp - the product formatter's thread scaling alone (no reader,
// no device): nsd_format_range_compact_fh over one resident batch of compact
// records (written by tools/fmtbench/prep.py), each thread formatting its
// parts into its own pre-touched buffer.  Development tool.
//   fmt_bench <dir> [pin] [pinned-input] [rotate-output]
#include <chrono>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <pthread.h>
#include <sched.h>
#include <string>
#include <thread>
#include <vector>

#include "../../include/netsniff_dissect.h"

static std::vector<char> rd(const std::string &p)
{
	FILE *f = fopen(p.c_str(), "rb");
	if (!f) {
		perror(p.c_str());
		exit(1);
	}
	fseek(f, 0, SEEK_END);
	const long n = ftell(f);
	fseek(f, 0, SEEK_SET);
	std::vector<char> v(n);
	if (fread(v.data(), 1, n, f) != (size_t)n)
		exit(1);
	fclose(f);
	return v;
}

int main(int argc, char **argv)
{
	const std::string d = argc > 1 ? argv[1] : ".";
	const bool pin = argc > 2 && atoi(argv[2]);
	const bool hm = argc > 3 && atoi(argv[3]);
	const bool rot = argc > 4 && atoi(argv[4]);
	auto fr0 = rd(d + "/frames.bin"), de0 = rd(d + "/desc.bin"), cr0 = rd(d + "/crec.bin"), po0 = rd(d + "/pool.bin"),
	     fh0 = rd(d + "/fh.bin");
	auto place = [&](std::vector<char> &v) -> char * {
		if (!hm)
			return v.data();
		void *p = nullptr;
		if (hipHostMalloc(&p, v.size(), hipHostMallocDefault) != hipSuccess)
			exit(2);
		memcpy(p, v.data(), v.size());
		return (char *)p;
	};
	char *fr = place(fr0), *de = place(de0), *cr = place(cr0), *po = place(po0), *fh = place(fh0);
	const uint32_t n = (uint32_t)(de0.size() / 8);
	cpu_set_t set;
	sched_getaffinity(0, sizeof(set), &set);
	std::vector<int> cpus;
	for (int c = 0; c < CPU_SETSIZE; c++)
		if (CPU_ISSET(c, &set))
			cpus.push_back(c);
	for (int rep = 0; rep < 2; rep++)
		for (int th : { 1, 2, 4, 8, 16 }) {
			const int parts = th * 4;
			std::vector<std::vector<char>> bufs(parts);
			for (auto &b : bufs) {
				b.resize((size_t)(n / parts + 1) * 700);
				memset(b.data(), 1, b.size());
			}
			double best = 1e30;
			for (int pass = 0; pass < (rot ? 4 : 1); pass++) {
			const auto t0 = std::chrono::steady_clock::now();
			std::vector<std::thread> ts;
			for (int t = 0; t < th; t++)
				ts.emplace_back([&, t]() {
					if (pin) {
						cpu_set_t one;
						CPU_ZERO(&one);
						CPU_SET(cpus[(size_t)(2 * t) % cpus.size()], &one);
						pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
					}
					for (int p = t; p < parts; p += th) {
						const int ob = rot ? (p + pass * 4) % parts : p;
						const uint32_t lo = (uint32_t)((uint64_t)n * p / parts), hi = (uint32_t)((uint64_t)n * (p + 1) / parts);
						const long r = nsd_format_range_compact_fh(
							(const uint8_t *)fr, (const nsd_desc_t *)de, nullptr,
							(const nsd_frame_hdr_t *)fh, 1, lo, hi, 1, 0, (const nsd_crec *)cr,
							(const uint32_t *)po, bufs[ob].data(), bufs[ob].size(), nullptr, nullptr);
						if (r < 0) {
							printf("format error %ld\n", r);
							exit(1);
						}
					}
				});
			for (auto &x : ts)
				x.join();
			const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
			best = dt < best ? dt : best;
			}
			printf("pin %d pinned-in %d rotate %d threads %d %.3f Mpkt/s\n", (int)pin, (int)hm, (int)rot, th,
			       n / best / 1e6);
		}
	return 0;
}
