/* nsd_bpf_oracle.h - TEST INFRASTRUCTURE ONLY: CPU restatement of
 * netsniff-ng's classic-BPF validator and userland interpreter (bpf.c), the
 * checker for the device filter (netsniff-ng_amd/csrc/nsd_bpf.hip). */
#ifndef NSD_BPF_ORACLE_H
#define NSD_BPF_ORACLE_H

#include <stdint.h>

#include "../include/netsniff_dissect.h"   /* nsd_bpf_insn (= struct sock_filter) */

#ifdef __cplusplus
extern "C" {
#endif

/* __bpf_validate (bpf.c:388-506): 1 = valid, 0 = not */
int nsor_bpf_validate(const nsd_bpf_insn *prog, uint32_t len);

/* bpf_run_filter (bpf.c:508-705) over pkt[0, plen) */
uint32_t nsor_bpf_run(const nsd_bpf_insn *prog, uint32_t len, const uint8_t *pkt, uint32_t plen);

/* the same over a batch of packed frames (desc as in netsniff_dissect.h) */
void nsor_bpf_batch(const nsd_bpf_insn *prog, uint32_t len, const uint8_t *frames,
		    const uint64_t *desc, uint32_t n, uint32_t *verdict);

#ifdef __cplusplus
}
#endif

#endif /* NSD_BPF_ORACLE_H */
