/*
 * entry_harness.c - netsniff-ng's `--in file.pcap` loop (read_pcap,
 * netsniff-ng.c:626-787) reduced to what the dissector surface sees, linked
 * against libnsdissect.so the way INTEGRATION.md links netsniff-ng:
 *
 *   dissector_init_all(mode)                      netsniff-ng.c:678
 *   per record: dissector_entry_point(buf, caplen, linktype, mode, &sll)
 *                                                 netsniff-ng.c:735
 *   dissector_cleanup_all()                       netsniff-ng.c:764
 *
 * The executable provides tprintf / tprintf_flush (as netsniff-ng's
 * tprintf.o does: the same 1 KiB buffer and wrap rules, into memory instead
 * of stdout), and the per-packet text ends are written beside it, so tests
 * compare them with the golden per-packet text.  Test infrastructure.
 *
 *   entry_harness -m MODE [-e ETCDIR] [-w COLS] [-r REPS] in.pcap out.txt out.ends
 *   -r REPS: timing mode (text discarded after every packet, the loop over
 *   all records repeated REPS times; prints "pkts=N us_per_pkt=X" on stdout)
 */
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../include/netsniff_dissect.h"

/* netsniff-ng's tprintf (tprintf.c:65-162), restated: a 1 KiB buffer,
 * flushed when a piece does not fit and by tprintf_flush, each flush wrapped
 * for a terminal `g_cols` wide (-w, default 65535 like nsref -w 65535); the
 * flushed text goes to tbuf */
static char *tbuf;
static size_t tlen, tcap;
static char buffer[1024];
static size_t buffer_use;
static int g_cols = 65535;
static long line_count;

static void put(char c)
{
	if (tlen + 1 > tcap) {
		tcap = tcap * 2 + 65536;
		tbuf = realloc(tbuf, tcap);
		if (!tbuf)
			abort();
	}
	tbuf[tlen++] = c;
}

static void flush_buffer(void)
{
	long term_len = g_cols - 5;
	size_t color_open = 0;
	for (size_t i = 0; i < buffer_use; ++i) {
		if (buffer[i] == '\n') {
			term_len = g_cols - 5;
			line_count = -1;
		}
		if (buffer[i] == 033 && i + 1 < buffer_use && buffer[i + 1] == '[')
			color_open++;
		if (color_open == 0 && line_count >= term_len) {
			put('\n');
			for (int k = 0; k < 3; k++)
				put(' ');
			line_count = 3;
			while (i < buffer_use && (buffer[i] == ' ' || buffer[i] == ','))
				i++;
		}
		if (color_open > 0 && buffer[i] == 'm')
			color_open--;
		put(buffer[i]);
		line_count++;
	}
	buffer_use = 0;
}

void tprintf(char *msg, ...)
{
	va_list vl;
	size_t avail = sizeof(buffer) - buffer_use;
	va_start(vl, msg);
	int ret = vsnprintf(buffer + buffer_use, avail, msg, vl);
	va_end(vl);
	if (ret < 0 || (size_t)ret > sizeof(buffer))
		abort();   /* the reference panics */
	if ((size_t)ret >= avail) {
		flush_buffer();
		va_start(vl, msg);
		ret = vsnprintf(buffer, sizeof(buffer), msg, vl);
		va_end(vl);
		if (ret < 0)
			abort();
	}
	buffer_use += ret;
}

static size_t flushes;
void tprintf_flush(void)
{
	flushes++;
	flush_buffer();
}

static uint32_t sw32(uint32_t v, int s) { return s ? __builtin_bswap32(v) : v; }

int main(int argc, char **argv)
{
	int mode = PRINT_NORM, reps = 0, c;
	const char *etc = "/nonexistent-netsniff-ng-etc";
	while ((c = getopt(argc, argv, "m:e:r:w:")) != -1) {
		if (c == 'm') mode = atoi(optarg);
		else if (c == 'w') g_cols = atoi(optarg);
		else if (c == 'e') etc = optarg;
		else if (c == 'r') reps = atoi(optarg);
		else return 2;
	}
	if (argc - optind < 1 || (!reps && argc - optind < 3))
		return 2;
	FILE *f = fopen(argv[optind], "rb");
	if (!f)
		return 3;
	fseek(f, 0, SEEK_END);
	long sz = ftell(f);
	fseek(f, 0, SEEK_SET);
	uint8_t *file = malloc(sz);
	if (fread(file, 1, sz, f) != (size_t)sz)
		return 3;
	fclose(f);
	uint32_t magic;
	memcpy(&magic, file, 4);
	int swapped = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
	uint32_t linktype;
	memcpy(&linktype, file + 20, 4);
	linktype = sw32(linktype, swapped);

	nsd_set_etcdir(etc);
	dissector_init_all(mode);

	/* records: 16-byte classic header, then caplen bytes */
	size_t nrec = 0, cap_recs = 1024;
	long *offs = malloc(cap_recs * sizeof(long));
	uint32_t *caps = malloc(cap_recs * sizeof(uint32_t));
	for (long o = 24; o + 16 <= sz;) {
		uint32_t caplen;
		memcpy(&caplen, file + o + 8, 4);
		caplen = sw32(caplen, swapped);
		if (nrec == cap_recs) {
			cap_recs *= 2;
			offs = realloc(offs, cap_recs * sizeof(long));
			caps = realloc(caps, cap_recs * sizeof(uint32_t));
		}
		offs[nrec] = o + 16;
		caps[nrec] = caplen;
		nrec++;
		o += 16 + caplen;
	}
	uint8_t *buf = malloc(1 << 20);
	struct { uint16_t family, protocol; int32_t ifindex; uint16_t hatype; uint8_t pkttype, halen, addr[8]; }
		sll;
	memset(&sll, 0, sizeof(sll));

	if (reps) {
		struct timespec t0, t1;
		clock_gettime(CLOCK_MONOTONIC, &t0);
		for (int r = 0; r < reps; r++) {
			for (size_t i = 0; i < nrec; i++) {
				memcpy(buf, file + offs[i], caps[i]);
				dissector_entry_point(buf, caps[i], (int)linktype, mode, (struct sockaddr_ll *)&sll);
				tlen = 0;   /* the text is written nowhere (/dev/null) */
			}
		}
		clock_gettime(CLOCK_MONOTONIC, &t1);
		double us = (t1.tv_sec - t0.tv_sec) * 1e6 + (t1.tv_nsec - t0.tv_nsec) / 1e3;
		printf("pkts=%zu us_per_pkt=%.4f\n", nrec * (size_t)reps, us / ((double)nrec * reps));
		dissector_cleanup_all();
		return 0;
	}

	FILE *ft = fopen(argv[optind + 1], "wb"), *fe = fopen(argv[optind + 2], "wb");
	if (!ft || !fe)
		return 4;
	for (size_t i = 0; i < nrec; i++) {
		/* read_pcap reads into a reused 1 MiB buffer (netsniff-ng.c:680);
		 * bytes past caplen are zero here (the parity domain) */
		memset(buf, 0, 4096);
		memcpy(buf, file + offs[i], caps[i]);
		size_t before = flushes;
		dissector_entry_point(buf, caps[i], (int)linktype, mode, (struct sockaddr_ll *)&sll);
		if (mode != PRINT_NONE && flushes != before + 1)
			return 5;   /* dissector.c:120: one flush per packet */
		uint64_t end = tlen;
		fwrite(&end, sizeof(end), 1, fe);
	}
	fwrite(tbuf, 1, tlen, ft);
	fclose(ft);
	fclose(fe);
	dissector_cleanup_all();
	return 0;
}
