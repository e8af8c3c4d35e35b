"""Timing-only experiment builds (not products): copy the product sources to a
scratch directory, apply text patches to clyscan.hip, and build
couloydb_amd/libexp_<name>.so.  Usage: python tools/xp_build.py NAME [NAME...]
with NAME one of the PATCHES below."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATCHES = {
    # no compact-entry stores (tuples come out wrong: timing only)
    "nocomp": [("    if (idx < CAP_T) __builtin_amdgcn_raw_buffer_store_b128(v, rs.trs, (int)(idx * 16u), 0, 0);",
                "    if (idx < CAP_T) { if (rs.g->walk_max == 12345678u) __builtin_amdgcn_raw_buffer_store_b128(v, rs.trs, (int)(idx * 16u), 0, 0); }")],
    # no segment-register stores
    "noseg": [("        if (m > 0)\n            __builtin_amdgcn_raw_buffer_store_b32(Rp, srs,",
               "        if (m > 0 && g->walk_max == 12345678u)\n            __builtin_amdgcn_raw_buffer_store_b32(Rp, srs,")],
    # no snapshot stores
    "nosnap": [("    if (r < CAP_T) __builtin_amdgcn_raw_buffer_store_b32(v, rs.trs, (int)(r * 16u + 4u), 0, 0);",
                "    if (r < CAP_T) { if (rs.g->walk_max == 12345678u) __builtin_amdgcn_raw_buffer_store_b32(v, rs.trs, (int)(r * 16u + 4u), 0, 0); }")],
}
PATCHES["nostore"] = PATCHES["nocomp"] + PATCHES["noseg"] + PATCHES["nosnap"]
# every kernel after k_scan returns at once: k_scan alone is timed, and no
# kernel reads what a patched k_scan left out (a garbled compact entry sent
# k_emit's header loads out of bounds once)
SCAN_ONLY = [("    if (guard >= 0 && g->nfix[guard] == 0) return;  // (device round: nothing was re-resolved)",
              "    if (g->walk_max != 12345678u) return;"),
             ("    if (g->nfix[slot] == 0) return;                        // (uniform: before the LDS setup's barrier)",
              "    if (g->walk_max != 12345678u) return;"),
             ("    if (g->nfix[slot] || g->spill_over || g->fail) return;   // the chain is not final yet (k_refix first) / run again / failed",
              "    if (g->walk_max != 12345678u) return;"),
             ("    if (g->nfix[slot] || g->spill_over || g->fail) return;   // k_emit did not run",
              "    if (g->walk_max != 12345678u) return;")]
for k in ("nocomp", "noseg", "nosnap", "nostore"):
    PATCHES[k] = PATCHES[k] + SCAN_ONLY
PATCHES["base"] = list(SCAN_ONLY)
# counters: blocks that reach the general pass, in-wave agreement rounds (stderr)
PATCHES["cnt"] = [
    ("""            if (!done) {
                // ---- general pass""", """            if (!done) {
                if (lane == 0) atomicAdd(&g->rounds, 1u);
                // ---- general pass"""),
    ("""        const u64 bm = __ballot(bad);
        if (!bm) return L;""", """        const u64 bm = __ballot(bad);
        if (!bm) return L;
        if (lane == 0) atomicAdd((unsigned long long*)&g->walk_dbg, 1ull);"""),
    ("""    float ms_scan = 0, ms_link = 0, ms_emit = 0, ms_fin = 0;""",
     """    fprintf(stderr, "xp: general-pass blocks %u, agreement rounds %llu\\n", c->h_g->rounds,
            (unsigned long long)c->h_g->walk_dbg);
    float ms_scan = 0, ms_link = 0, ms_emit = 0, ms_fin = 0;"""),
]
# the stride round repeated while it takes a full 64 records and the chain stays in the block
PATCHES["sloop"] = [
    ("""                if (S.ref_ok) stride_round<BM>(F, S, tb, bs, stg, smem, cl, K4, rs, lane, mk);""",
     """                for (int sr = 0; sr < 8 && S.ref_ok; sr++) {
                    const uint32_t c1 = S.tcnt;
                    stride_round<BM>(F, S, tb, bs, stg, smem, cl, K4, rs, lane, mk);
                    if (S.tcnt - c1 < 64u || S.dead || S.X >= bs + CLY_BLK) break;
                }"""),
]
# section clocks of tile_body (s_memtime, summed over waves) and general-pass counts (stderr)
PATCHES["prof"] = [
    ("""    uint32_t run_next;           // k_scan's run counter (runs past the grid's first one each)
};""", """    uint32_t run_next;           // k_scan's run counter (runs past the grid's first one each)
    unsigned long long xp_t[8];
};"""),
    ("""    uint32_t Rp = 0;             // the previous block's segment register (stored at the next block's top)""",
     """    uint32_t Rp = 0;             // the previous block's segment register (stored at the next block's top)
    unsigned long long xt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tq = __builtin_amdgcn_s_memtime();
#define XPT(k) { const unsigned long long tn_ = __builtin_amdgcn_s_memtime(); xt[k] += tn_ - tq; tq = tn_; }"""),
    ("""            if (S.X == NONE32) S.X = guess_entry(F, bs, stg, hc, lane);    // the tile's guessed entry
            bool done = true;""", """            XPT(6)
            if (S.X == NONE32) S.X = guess_entry(F, bs, stg, hc, lane);    // the tile's guessed entry
            XPT(0)
            bool done = true;"""),
    ("""            if (!done) {
                // ---- general pass""", """            XPT(1)
            if (!done) {
                xt[7]++;
                // ---- general pass"""),
    ("""                {
                    L = seg_resolve(K, L, lane, X, g);""", """                XPT(2)
                {
                    L = seg_resolve(K, L, lane, X, g);
                    XPT(3)"""),
    ("""        {
            // bytes from the terminal on read as zero""", """        XPT(4)
        {
            // bytes from the terminal on read as zero"""),
    ("""            carry = S.carry_next; cmark = S.cmark_next;
            S.carry_next = 0; S.cmark_next = false;
        }""", """            carry = S.carry_next; cmark = S.cmark_next;
            S.carry_next = 0; S.cmark_next = false;
        }
        XPT(5)"""),
    ("""    if (lane == 0) {
        ctab[CH_NWORD] = S.nch_have;""", """    if (lane == 0) for (int k = 0; k < 8; k++) atomicAdd(&g->xp_t[k], xt[k]);
    if (lane == 0) {
        ctab[CH_NWORD] = S.nch_have;"""),
    ("""        const u64 bm = __ballot(bad);
        if (!bm) return L;""", """        const u64 bm = __ballot(bad);
        if (!bm) { if (lane == 0 && iter) atomicAdd((unsigned long long*)&g->walk_dbg, (unsigned long long)iter << 40); return L; }"""),
    ("""    float ms_scan = 0, ms_link = 0, ms_emit = 0, ms_fin = 0;""",
     """    fprintf(stderr, "xp: guess %llu pred %llu gen-walk %llu resolve %llu gen-out %llu crc %llu stage %llu | general blocks %llu resolve iters %llu\\\\n",
            c->h_g->xp_t[0], c->h_g->xp_t[1], c->h_g->xp_t[2], c->h_g->xp_t[3], c->h_g->xp_t[4], c->h_g->xp_t[5],
            c->h_g->xp_t[6], c->h_g->xp_t[7], (unsigned long long)(c->h_g->walk_dbg >> 40));
    float ms_scan = 0, ms_link = 0, ms_emit = 0, ms_fin = 0;"""),
]
# every tile's loads read its part's first tile (L2-resident): k_scan's time with
# the HBM latency taken out, same record work (timing only)
PATCHES["l2"] = [
    ("""    const uint32_t off = bs + 64u * (uint32_t)(lane & 15) + 16u * (uint32_t)(lane >> 4);""",
     """    const uint32_t off = (bs & (CLY_TILE - 1u)) + 64u * (uint32_t)(lane & 15) + 16u * (uint32_t)(lane >> 4);"""),
    ("""    if (lane < 2) hl = load16z(base, (uint64_t)bs + CLY_BLK + 16 * lane, flen);""",
     """    if (lane < 2) hl = load16z(base, (uint64_t)((bs + CLY_BLK) & (CLY_TILE - 1u)) + 16 * lane, flen);"""),
] + SCAN_ONLY
# blocks after two general-pass blocks in a row skip the predictive walk (every
# 8th tries it again)
PATCHES["pskip"] = [
    ("""    bool ref_ok;
""", """    bool ref_ok;
    uint32_t gp_run;
"""),
    ("""    S.ref_ok = false; S.ref_s = 0;""", """    S.gp_run = 0; S.ref_ok = false; S.ref_s = 0;"""),
    ("""                done = pred_walk<BM>(F, S, tb, bs, stg, smem, cl, K4, rs, lane, mk);
                if (S.tcnt != c0) stride_ref(F, S, bs, stg);
            }""", """                if (S.gp_run >= 2 && (S.gp_run & 7u) != 0) {
                    const uint64_t Xs = S.X, be = (uint64_t)bs + CLY_BLK;
                    done = S.dead || !(Xs < be || (Xs == F.len && F.len == be));
                } else done = pred_walk<BM>(F, S, tb, bs, stg, smem, cl, K4, rs, lane, mk);
                if (S.tcnt != c0) stride_ref(F, S, bs, stg);
            }
            S.gp_run = done ? 0u : S.gp_run + 1u;"""),
]
PATCHES["gp1"] = [("#define GP_TRIES 2 ", "#define GP_TRIES 1 ")]
PATCHES["gp3"] = [("#define GP_TRIES 2 ", "#define GP_TRIES 3 ")]
PATCHES["sloopcnt"] = PATCHES["sloop"] + PATCHES["cnt"]
PATCHES["run1"] = [("#define RUN_TILES 4", "#define RUN_TILES 1")]
PATCHES["run8"] = [("#define RUN_TILES 4", "#define RUN_TILES 8")]
PATCHES["run16"] = [("#define RUN_TILES 4", "#define RUN_TILES 16")]


def build(name):
    """NAME: a PATCHES key applied to the working tree, or git:<commit> (that
    commit's sources as they are; the library is libexp_<commit>.so)."""
    tmp = tempfile.mkdtemp(prefix="clyxp_")
    try:
        if name.startswith("git:"):
            commit = name[4:]
            ar = subprocess.run(["git", "-C", ROOT, "archive", commit, "couloydb_amd/csrc", "include"],
                                check=True, capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", tmp], input=ar, check=True)
            name, patches = commit, []
        else:
            shutil.copytree(os.path.join(ROOT, "couloydb_amd", "csrc"), os.path.join(tmp, "couloydb_amd", "csrc"))
            shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
            patches = PATCHES[name]
        p = os.path.join(tmp, "couloydb_amd", "csrc", "clyscan.hip")
        s = open(p).read()
        for old, new in patches:
            assert s.count(old) == 1, (name, old[:60])
            s = s.replace(old, new)
        open(p, "w").write(s)
        out = os.path.join(ROOT, "couloydb_amd", "libexp_%s.so" % name)
        srcs = [f for f in ["clyscan.hip", "clymerge.hip", "clyindex.hip", "clyload.hip", "clyorder.hip"]
                if os.path.exists(os.path.join(os.path.dirname(p), f))]
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                               "-w", "-DCLY_SRC_HASH=\"xp-%s\"" % name, "-o", out] + srcs,
                              cwd=os.path.dirname(p))
        print("built", out)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(4) as ex:
        list(ex.map(build, sys.argv[1:]))
