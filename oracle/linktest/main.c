/*
 * oracle/linktest/main.c -- host-side driver of kat_kernel.c (TEST
 * INFRASTRUCTURE ONLY).  Runs the kernel-side KATs, which call libmicksum's
 * in_cksum* through the reference's own <machine/in_cksum.h> declarations,
 * and compares with the values SURVEY.md 8(a) records from the compiled
 * reference.  Prints one JSON line; exit status 0 iff every value matches.
 */
#include <stdio.h>
#include <stdlib.h>

extern int mi_link_kats(void);
/* libmicksum's own symbols (include/mi_cksum.h): which mode served the
 * drop-ins, and how many GPU-mode calls an error sent to the host fold. */
extern int mi_cksum_set_dropin_mode(int mode);
extern unsigned long long mi_cksum_dropin_degraded(void);
extern unsigned int mi_link_got[];

static const struct {
	const char *name;
	unsigned int want;
} kat[] = {
	{"KAT1 rfc1071", 0x0d22},         {"KAT2 hdr aligned", 0x61b8},
	{"KAT3 hdr 2mod4", 0x61b8},       {"KAT4 hdr odd", 0xb861},
	{"KAT5 zeros", 0xffff},           {"KAT6 ones", 0x0000},
	{"KAT7 len1", 0xffff},            {"KAT7 len2", 0xfeff},
	{"KAT7 len3", 0xfefd},            {"KAT7 len63", 0x3b1c},
	{"KAT7 len64", 0xfc1b},           {"KAT7 len1500", 0x4e39},
	{"KAT7 len1501", 0x4d5d},         {"KAT7 len9000", 0xb739},
	{"KAT7 len65535", 0x3ec1},        {"KAT7 len65536", 0x3fc0},
	{"KAT7b len1", 0xfffe},           {"KAT7b len64", 0xdbfb},
	{"KAT7b len1500", 0x5d4d},        {"KAT7b len9000", 0x11b7},
	{"KAT7b len65536", 0xc03f},       {"KAT8 pseudo tcp", 0x900a},
	{"KAT9 pseudo udp", 0xa1ed},      {"KAT10 in_pseudo", 0x2289},
	{"KAT11 chain odd", 0x4e39},      {"KAT12 skip20", 0xb293},
	{"addword carry", 0x0001},        {"addword", 0x5555},
};

int
main(void)
{
	int n = mi_link_kats(), bad = 0, i;
	int nk = (int)(sizeof(kat) / sizeof(kat[0]));

	if (n != nk) {
		printf("{\"error\": \"ran %d results, expected %d\"}\n", n, nk);
		return 2;
	}
	printf("{\"kats\": %d, \"results\": {", nk);
	for (i = 0; i < nk; i++) {
		int ok = mi_link_got[i] == kat[i].want;
		bad += !ok;
		printf("%s\"%s\": [\"0x%04x\", \"0x%04x\", %s]", i ? ", " : "", kat[i].name, mi_link_got[i],
		       kat[i].want, ok ? "true" : "false");
	}
	{
		int mode = mi_cksum_set_dropin_mode(0);
		mi_cksum_set_dropin_mode(mode);
		printf("}, \"failed\": %d, \"mode\": \"%s\", \"degraded\": %llu}\n", bad,
		       mode == 1 ? "gpu" : "host", mi_cksum_dropin_degraded());
	}
	return bad ? 1 : 0;
}
