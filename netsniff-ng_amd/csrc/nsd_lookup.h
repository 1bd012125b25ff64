// nsd_lookup.h - id -> name tables of the reference's lookup.c
// (udp.conf / tcp.conf / ether.conf / oui.conf under ETCDIRE_STRING).
#pragma once
#include <stdint.h>

namespace nsd {
const char *lookup_port_udp(uint32_t id);
const char *lookup_port_tcp(uint32_t id);
const char *lookup_ether_type(uint32_t id);
const char *lookup_vendor(uint32_t id);
// load the four tables from dir as dissector_init_all does (messages on stderr)
int lookup_init_reporting(const char *dir);
}
