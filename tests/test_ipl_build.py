"""The LDS IP-table builder (retina_amd/csrc/ipl_build.h), compiled host-only with g++:
every endpoint IP is found with its slot by the host mirror of the kernel probe, absent
IPs miss, and pod-IP sets up to the C2 size (10k pods, ~10.5k IPs) fit the image budget."""

import os
import subprocess

import numpy as np
import pytest

from retina_amd import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("ipl") / "ipl_build_test")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "retina_amd", "csrc"),
                    os.path.join(ROOT, "tests", "ipl_build_test.cpp"), "-o", exe], check=True)
    return exe


def run_sets(exe, sets):
    lines = [str(len(sets))]
    for ents in sets:
        lines.append(str(len(ents)))
        lines.extend("%d %d" % (ip, sl) for ip, sl in ents)
    out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True).stdout.split("\n")
    res = []
    for ln in out:
        if ln.strip():
            (built, nb, seed, nbytes, load, found, absent, rbuilt, npfx, nblk, rbytes, rfound, rabsent,
             dbuilt, dnblk, dbytes, dfound, dabsent) = ln.split()
            res.append(dict(built=int(built), nb=int(nb), bytes=int(nbytes), load=float(load),
                            found=int(found), absent=int(absent), rbuilt=int(rbuilt), npfx=int(npfx),
                            nblk=int(nblk), rbytes=int(rbytes), rfound=int(rfound), rabsent=int(rabsent),
                            dbuilt=int(dbuilt), dnblk=int(dnblk), dbytes=int(dbytes), dfound=int(dfound),
                            dabsent=int(dabsent)))
    return res


def pod_sets():
    sets = []
    for npods in (1, 7, 400, 2_000, 10_000):
        p = W.make_pods(npods, seed=npods)
        sets.append([(int(ip), int(o)) for ip, o in zip(p.ips, p.ip_owner)])
    rng = np.random.default_rng(5)
    ips = np.unique(rng.integers(0, 2**32 - 1, 12_000, dtype=np.uint64)).astype(np.uint32)
    sets.append([(int(ip), i % 60_000) for i, ip in enumerate(ips)])           # random IPs
    sets.append([(0x0A000000 + i, i) for i in range(9_000)])                    # sequential BE
    return sets


def test_builder_finds_every_key(harness):
    sets = pod_sets()
    for ents, r in zip(sets, run_sets(harness, sets)):
        assert r["built"] == 1, (len(ents), r)
        assert r["found"] == len(ents)
        assert r["absent"] > 99_000
        assert r["bytes"] <= 112 * 1024


def test_builder_refuses_unimageable(harness):
    too_many = [(0x0A000000 + i, i % 1000) for i in range(40_000)]   # > image budget
    bad_slot = [(1, 0xFFFF)]                                         # slot id reserved
    bad_key = [(0xFFFFFFFF, 3)]                                      # empty-key marker
    r = run_sets(harness, [too_many, bad_slot, bad_key])
    assert [x["built"] for x in r] == [0, 0, 0]


def test_radix_image_matches(harness):
    """The radix image (pod IPs in <= 4 /16 prefixes): every key found with its slot,
    absent IPs -- random and next to pod IPs -- miss; C2's 10k pods take ~80 /24 blocks."""
    sets = pod_sets()
    res = run_sets(harness, sets)
    for ents, r in zip(sets, res):
        if not r["rbuilt"]:
            continue
        assert r["rfound"] == len(ents)
        assert r["rabsent"] == 0  # no absent IP resolves to a slot
        assert r["rbytes"] <= 112 * 1024
    c2 = res[4]  # make_pods(10_000): 10.0.x.x primaries + 10.128.x.x secondaries
    assert c2["rbuilt"] == 1 and c2["npfx"] == 2 and 70 <= c2["nblk"] <= 80
    assert res[5]["rbuilt"] == 0  # random IPs: far more than 4 prefixes
    # more than 4 prefixes, or a reserved slot id, refuse
    r = run_sets(harness, [[(0x0A00 + k | (i << 24), i) for k in range(5) for i in range(3)], [(1, 0xFFFF)]])
    assert [x["rbuilt"] for x in r] == [0, 0]


def test_dense_radix_image_matches(harness):
    """The dense radix image (each prefix's /24s one run of third octets, no row table):
    every key found with its slot, absent IPs -- random, next to pod IPs, and in the
    pods' /16s outside their /24 runs -- miss; C2's 10k pods: 2 runs of <= 40 /24s."""
    sets = pod_sets()
    res = run_sets(harness, sets)
    for ents, r in zip(sets, res):
        if not r["dbuilt"]:
            continue
        assert r["dfound"] == len(ents)
        assert r["dabsent"] == 0
        assert r["dbytes"] <= 112 * 1024
    c2 = res[4]
    assert c2["dbuilt"] == 1 and 78 <= c2["dnblk"] <= 80 and c2["dbytes"] == (c2["dnblk"] + 1) * 512
    assert res[5]["dbuilt"] == 0  # random IPs: far more than 4 prefixes
    # a run with holes gets empty blocks for them; a run too long for the budget refuses
    holes = [(0x0A0A | (o3 << 16) | (7 << 24), o3) for o3 in (3, 9, 200)]
    wide = [(0x0A0A | (o3 << 16) | (k << 24), o3 * 256 + k) for o3 in range(256) for k in (1, 2)] + \
           [(0x0B0A | (o3 << 16) | (1 << 24), 7) for o3 in range(0, 256, 2)]
    r = run_sets(harness, [holes, wide])
    assert r[0]["dbuilt"] == 1 and r[0]["dnblk"] == 198 and r[0]["dfound"] == 3 and r[0]["dabsent"] == 0
    assert r[1]["dbuilt"] == 0  # 512 blocks of 512 B: more than 112 KiB
