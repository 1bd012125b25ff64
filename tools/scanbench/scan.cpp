// scan.cpp - a mapped pcap-like file's serial header walk (the replay
// reader's scan_batch) under page-table and prefetch variants: 0 plain,
// 1 MAP_POPULATE, 2 prefetch PD bytes ahead, 3 pages populated by 4 threads,
// 4 = 2 + 3.  Development tool.  Usage: scan DIR mk; scan DIR <variant>
#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <cstdint>
#include <thread>
#include <vector>
#include <string>
#ifndef PD
#define PD 4096
#endif
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char **argv) {
	const std::string path_s = std::string(argv[1]) + "/f.bin"; const char *path = path_s.c_str();
	const size_t N = 4u << 20;
	if (argc > 2 && !strcmp(argv[2], "mk")) { FILE *f = fopen(path, "wb"); std::vector<uint8_t> r(80, 0); uint32_t cl = 64; memcpy(&r[8], &cl, 4); memcpy(&r[12], &cl, 4); fwrite("0123456789abcdefghijklmn", 1, 24, f); for (size_t i = 0; i < N; i++) fwrite(r.data(), 1, 80, f); fclose(f); return 0; }
	int variant = atoi(argv[2]);
	int fd = open(path, O_RDONLY); struct stat sb; fstat(fd, &sb);
	double t0 = now();
	int fl = MAP_PRIVATE | (variant == 1 ? MAP_POPULATE : 0);
	uint8_t *m = (uint8_t *)mmap(nullptr, sb.st_size, PROT_READ, fl, fd, 0);
	madvise(m, sb.st_size, MADV_SEQUENTIAL);
	double t1 = now();
	std::vector<std::thread> th;
	if (variant == 3 || variant == 4) {
		const size_t chunk = 8 << 20;
		for (int t = 0; t < 4; t++) th.emplace_back([=] { for (size_t o = (size_t)t * chunk; o < (size_t)sb.st_size; o += 4 * chunk) { size_t l = std::min(chunk, (size_t)sb.st_size - o); madvise(m + o, l, MADV_POPULATE_READ); } });
	}
	size_t pos = 24, n = 0;
	while (pos + 16 <= (size_t)sb.st_size) {
		uint32_t cl; memcpy(&cl, m + pos + 8, 4);
		if (variant == 2 || variant == 4) __builtin_prefetch(m + pos + PD);
		pos += 16 + cl; n++;
	}
	double t2 = now();
	for (auto &t : th) t.join();
	printf("variant %d: mmap %.1f ms, scan %.1f ms (%zu recs)\n", variant, (t1 - t0) * 1e3, (t2 - t1) * 1e3, n);
	return 0;
}
