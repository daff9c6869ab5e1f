"""Semantics of the generated cgroup-v2 device programs (gm_bpf_dev_build in native/src/gm_host.cpp),
executed with the Python eBPF interpreter against a reference model of the device-rule rules."""
import ctypes as C
import itertools
import struct

from hypothesis import given, settings
from hypothesis import strategies as st

from gpumounter_amd import _native
from gpumounter_amd.node import bpfvm
from gpumounter_amd.node.cgroup import _rule_array

TYPES = {"c": bpfvm.BPF_DEVCG_DEV_CHAR, "b": bpfvm.BPF_DEVCG_DEV_BLOCK}


def build(rules, default_allow=0, chain=-1):
    arr = _rule_array([_native.DevRule(t.encode(), acc, allow, 0, ma, mi)
                       for t, acc, allow, ma, mi in rules])
    lib = _native.host()
    need = -lib.gm_bpf_dev_build(arr, len(rules), default_allow, chain, None, 0)
    buf = (C.c_uint64 * need)()
    n = lib.gm_bpf_dev_build(arr, len(rules), default_allow, chain, buf, need)
    assert n == need
    return [int(buf[i]) for i in range(n)]


def model(rules, default_allow, dev_type, access, major, minor, chained=None):
    for t, acc, allow, ma, mi in rules:
        if t != "a" and TYPES[t] != dev_type:
            continue
        if access & ~acc & 7:
            continue
        if ma >= 0 and ma != major:
            continue
        if mi >= 0 and mi != minor:
            continue
        return allow
    if chained is not None:
        return chained(dev_type, access, major, minor)
    return default_allow


def test_simple_allow_list():
    rules = [("c", 6, 1, 226, 128), ("c", 6, 1, 226, 0), ("c", 6, 1, 511, 0)]
    prog = build(rules)
    assert bpfvm.run(prog, 2, 6, 226, 128) == 1
    assert bpfvm.run(prog, 2, 2, 226, 0) == 1          # read ⊂ rw
    assert bpfvm.run(prog, 2, 1, 226, 128) == 0        # mknod not granted
    assert bpfvm.run(prog, 2, 6, 226, 129) == 0        # another GPU
    assert bpfvm.run(prog, 1, 6, 226, 128) == 0        # block device with same numbers


def test_chained_program_falls_through_to_runtime_policy():
    prog = build([("c", 6, 1, 226, 130)], chain=-2)
    ch = bpfvm.runtime_default
    assert bpfvm.run(prog, 2, 6, 226, 130, ch) == 1    # ours
    assert bpfvm.run(prog, 2, 6, 1, 3, ch) == 1        # /dev/null from the runtime program
    assert bpfvm.run(prog, 2, 6, 226, 131, ch) == 0    # not granted anywhere
    assert bpfvm.run(prog, 2, 1, 8, 0, ch) == 1        # runtime allows mknod of anything
    # with the tail-call slot empty the program denies (fails closed)
    assert bpfvm.run(prog, 2, 6, 1, 3, None) == 0


def test_default_allow_without_chain_keeps_unrestricted_cgroup():
    prog = build([("c", 6, 0, 226, 131)], default_allow=1)
    assert bpfvm.run(prog, 2, 6, 226, 131) == 0
    assert bpfvm.run(prog, 2, 6, 226, 132) == 1


def test_wildcards_and_first_match_wins():
    rules = [("c", 6, 0, 226, 129), ("c", 7, 1, 226, -1), ("a", 1, 1, -1, -1)]
    prog = build(rules)
    assert bpfvm.run(prog, 2, 6, 226, 129) == 0   # explicit deny before the wildcard
    assert bpfvm.run(prog, 2, 7, 226, 200) == 1
    assert bpfvm.run(prog, 1, 1, 8, 1) == 1       # 'a' mknod wildcard
    assert bpfvm.run(prog, 1, 2, 8, 1) == 0


def test_exhaustive_against_model_small_grid():
    rules = [("c", 6, 1, 226, 128), ("b", 2, 1, 8, -1), ("c", 1, 0, -1, -1),
             ("c", 7, 1, 511, 0)]
    prog = build(rules, chain=-2)
    ch = bpfvm.runtime_default
    for dt, acc, ma, mi in itertools.product((1, 2), range(1, 8), (1, 8, 226, 511),
                                             (0, 3, 128, 129)):
        assert bpfvm.run(prog, dt, acc, ma, mi, ch) == model(rules, 0, dt, acc, ma, mi, ch), \
            (dt, acc, ma, mi)


rule_st = st.tuples(st.sampled_from(["c", "b", "a"]), st.integers(1, 7), st.integers(0, 1),
                    st.sampled_from([-1, 1, 226, 511]), st.sampled_from([-1, 0, 128, 129]))


@settings(max_examples=60, deadline=None)
@given(st.lists(rule_st, max_size=6), st.integers(0, 1), st.sampled_from([1, 2]),
       st.integers(1, 7), st.sampled_from([1, 226, 511, 7]), st.sampled_from([0, 128, 129, 5]))
def test_random_rule_sets_match_model(rules, default_allow, dt, acc, ma, mi):
    prog = build(rules, default_allow=default_allow)
    assert bpfvm.run(prog, dt, acc, ma, mi) == model(rules, default_allow, dt, acc, ma, mi)


def test_build_rejects_bad_input():
    lib = _native.host()
    bad = _rule_array([_native.DevRule(b"x", 6, 1, 0, 1, 1)])
    assert lib.gm_bpf_dev_build(bad, 1, 0, -1, None, 0) == -22
    # too-small buffer reports the needed size
    good = _rule_array([_native.DevRule(b"c", 6, 1, 0, 1, 1)])
    need = -lib.gm_bpf_dev_build(good, 1, 0, -1, None, 0)
    buf = (C.c_uint64 * 2)()
    assert lib.gm_bpf_dev_build(good, 1, 0, -1, buf, 2) == -need


def _as_xlated(prog):
    """Rewrite bpf_tail_call (call imm 12) the way the verifier does (BPF_JMP|BPF_TAIL_CALL)."""
    out = []
    for insn in prog:
        code, dst, src, off, imm = bpfvm.decode(insn)
        if code == 0x85 and imm == 12:
            insn = struct.unpack("<Q", struct.pack("<BBhi", 0xF5, 0, 0, 0))[0]
        out.append(insn)
    return out


def test_program_allows_reads_grants_back_from_raw_and_xlated_code():
    from gpumounter_amd.models.device import DeviceNode
    from gpumounter_amd.node.cgroup import build_program, program_allows
    nodes = [DeviceNode("/dev/dri/renderD130", 226, 130), DeviceNode("/dev/dri/card2", 226, 2),
             DeviceNode("/dev/kfd", 511, 0)]
    prog = build_program(nodes, chained=True)
    want = {(226, 130), (226, 2), (511, 0)}
    gpu_keys = {(226, m) for m in range(256)} | {(511, 0)}
    for p in (prog, _as_xlated(prog)):
        assert program_allows(p) & gpu_keys == want


# ------------------------------------------------------------------ set-mode program
def build_set(base=(), default_allow=0, chain=-1):
    arr = _rule_array([_native.DevRule(t.encode(), acc, allow, 0, ma, mi)
                       for t, acc, allow, ma, mi in base])
    lib = _native.host()
    need = -lib.gm_bpf_dev_build_set(-2, arr, len(base), default_allow, chain, None, 0)
    buf = (C.c_uint64 * need)()
    n = lib.gm_bpf_dev_build_set(-2, arr, len(base), default_allow, chain, buf, need)
    assert n == need
    return [int(buf[i]) for i in range(n)]


SET_KEYS = st.tuples(st.sampled_from([bpfvm.BPF_DEVCG_DEV_CHAR, bpfvm.BPF_DEVCG_DEV_BLOCK]),
                     st.sampled_from([1, 226, 511]), st.sampled_from([0, 3, 128, 130]))


@settings(max_examples=150, deadline=None)
@given(entries=st.dictionaries(SET_KEYS, st.integers(1, 7), max_size=6),
       dev_type=st.sampled_from([bpfvm.BPF_DEVCG_DEV_CHAR, bpfvm.BPF_DEVCG_DEV_BLOCK]),
       access=st.integers(1, 7), major=st.sampled_from([1, 226, 511, 7]),
       minor=st.sampled_from([0, 3, 128, 130, 9]), chained=st.booleans(),
       default_allow=st.integers(0, 1))
def test_set_program_matches_the_set_semantics(entries, dev_type, access, major, minor, chained,
                                               default_allow):
    """An access is allowed iff {type, major, minor} is in the allow set with every requested
    access bit; otherwise the runtime's chained program decides (or the default verdict). The
    program is the same whatever the set holds."""
    prog = build_set(default_allow=default_allow, chain=-2 if chained else -1)
    got = bpfvm.run(prog, dev_type, access, major, minor,
                    chained=bpfvm.runtime_default if chained else None, maps={0: entries})
    acc = entries.get((dev_type, major, minor))
    if acc is not None and access & ~acc == 0:
        want = 1
    elif chained:
        want = bpfvm.runtime_default(dev_type, access, major, minor)
    else:
        want = default_allow
    assert got == want


def test_set_program_with_lost_chain_compiles_the_base_list_in():
    base = [("c", 7, 1, 1, 3), ("c", 1, 1, -1, -1)]      # /dev/null rwm; mknod of any char
    prog = build_set(base=base, default_allow=0, chain=-1)
    table = {(bpfvm.BPF_DEVCG_DEV_CHAR, 226, 128): 6}
    rw = bpfvm.ACC_READ | bpfvm.ACC_WRITE
    assert bpfvm.run(prog, bpfvm.BPF_DEVCG_DEV_CHAR, rw, 226, 128, maps={0: table}) == 1
    assert bpfvm.run(prog, bpfvm.BPF_DEVCG_DEV_CHAR, rw, 1, 3, maps={0: table}) == 1   # base
    assert bpfvm.run(prog, bpfvm.BPF_DEVCG_DEV_CHAR, bpfvm.ACC_MKNOD, 226, 129,
                     maps={0: table}) == 1                                          # base mknod
    assert bpfvm.run(prog, bpfvm.BPF_DEVCG_DEV_CHAR, rw, 226, 129, maps={0: table}) == 0
    # length: one lookup whatever the set, versus one block per device for a straight line
    assert len(build_set()) < len(build([("c", 6, 1, 226, 128 + i) for i in range(4)]))
