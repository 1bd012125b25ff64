// nsd_lookup.cpp - name tables with the reference's loading semantics
// (lookup.c:33-95): lines read with fgets(128), id = strtol(, 0), name after
// ", " with trailing '\n' and ' ' stripped (str.c:75-90); a later line with
// the same id shadows an earlier one (lookup.c:84-88 prepends, :130-138
// returns the first match).  Ports / ether types: direct 64 Ki tables;
// OUI: sorted vector + binary search.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "../../include/netsniff_dissect.h"
#include "nsd_lookup.h"

namespace nsd {

static std::vector<std::string> t_udp, t_tcp, t_eth;   // "" = absent
static std::vector<std::pair<uint32_t, std::string>> t_oui;

static void strtrim_right(char *p, char c)
{
	size_t len = strlen(p);
	while (len && p[len - 1] == c)
		p[--len] = 0;
}

static int load(const std::string &path, int which)
{
	FILE *fp = fopen(path.c_str(), "r");
	char buff[128];
	std::vector<std::pair<uint32_t, std::string>> oui;
	if (!fp)
		return 0;
	std::vector<std::string> *tab = which == 0 ? &t_udp : which == 1 ? &t_tcp : which == 2 ? &t_eth : nullptr;
	if (tab)
		tab->assign(65536, std::string());
	memset(buff, 0, sizeof(buff));
	while (fgets(buff, sizeof(buff), fp)) {
		char *end, *ptr = buff;
		buff[sizeof(buff) - 1] = 0;
		unsigned id = (unsigned)strtol(ptr, &end, 0);
		if (id == 0 && end == ptr)
			continue;
		ptr = strstr(buff, ", ");
		if (!ptr)
			continue;
		ptr += 2;
		strtrim_right(ptr, '\n');
		strtrim_right(ptr, ' ');
		if (tab) {
			if (id < 65536)
				(*tab)[id] = ptr;
		} else if (id <= 0xFFFFFF) {
			oui.emplace_back(id, ptr);
		}
		memset(buff, 0, sizeof(buff));
	}
	fclose(fp);
	if (!tab) {
		// keep the last line per id
		std::stable_sort(oui.begin(), oui.end(),
				 [](const auto &a, const auto &b) { return a.first < b.first; });
		t_oui.clear();
		for (auto &e : oui) {
			if (!t_oui.empty() && t_oui.back().first == e.first)
				t_oui.back() = e;
			else
				t_oui.push_back(e);
		}
	}
	return 1;
}

static const char *get(const std::vector<std::string> &t, uint32_t id)
{
	if (id >= t.size() || t[id].empty())
		return nullptr;
	return t[id].c_str();
}

const char *lookup_port_udp(uint32_t id) { return get(t_udp, id); }
const char *lookup_port_tcp(uint32_t id) { return get(t_tcp, id); }
const char *lookup_ether_type(uint32_t id) { return get(t_eth, id); }
const char *lookup_vendor(uint32_t id)
{
	auto it = std::lower_bound(t_oui.begin(), t_oui.end(), id,
				   [](const auto &a, uint32_t v) { return a.first < v; });
	if (it == t_oui.end() || it->first != id)
		return nullptr;
	return it->second.c_str();
}

} // namespace nsd

extern "C" void nsd_lookup_cleanup(void)
{
	nsd::t_udp.clear();
	nsd::t_tcp.clear();
	nsd::t_eth.clear();
	nsd::t_oui.clear();
}

// dissector_init_ethernet's four lookup_init calls (dissector_eth.c:71-74,
// lookup.c:33-56): a missing file leaves its table empty, with the
// reference's message on stderr
int nsd::lookup_init_reporting(const char *dir)
{
	static const char *files[4] = { "udp.conf", "tcp.conf", "ether.conf", "oui.conf" };
	int n = 0;
	nsd_lookup_cleanup();
	for (int i = 0; i < 4; i++) {
		const std::string path = std::string(dir ? dir : "") + "/" + files[i];
		errno = 0;
		if (nsd::load(path, i))
			n++;
		else
			fprintf(stderr, "Cannot open %s: %s.Port name resolution won't be available.\n", path.c_str(),
				strerror(errno ? errno : ENOENT));
	}
	return n;
}

extern "C" int nsd_lookup_init(const char *dir)
{
	static const char *files[4] = { "udp.conf", "tcp.conf", "ether.conf", "oui.conf" };
	int n = 0;
	nsd_lookup_cleanup();
	if (!dir)
		return 0;
	for (int i = 0; i < 4; i++)
		n += nsd::load(std::string(dir) + "/" + files[i], i);
	return n;
}
