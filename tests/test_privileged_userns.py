"""Device nodes for containers in their own user namespace (root with mount + bpf; GM_PRIVILEGED_TESTS=0/1 forces off/on, root).

Runs tests/priv_userns_driver.py in a private mount namespace; see its docstring.
"""
import json
import os
import subprocess
import sys

import pytest
from conftest import privileged_skip

pytestmark = [pytest.mark.privileged, privileged_skip()]

HERE = os.path.dirname(os.path.abspath(__file__))


def test_userns_tenant_gets_openable_bind_mounted_nodes():
    r = subprocess.run(["unshare", "-m", "--propagation", "private", sys.executable,
                        os.path.join(HERE, "priv_userns_driver.py")],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-4000:]
    o = json.loads(r.stdout.strip().splitlines()[-1])
    # the reference's mknod: present by a plain read-back, yet the tenant cannot open it
    assert o["mknod_result"] == [0] and o["mknod_present"] == [True]
    assert o["mknod_tenant_open"] is False
    # bind mode, chosen because the tenant is in another user namespace
    assert o["bind_detected"] is True
    assert o["bind_present_before"] == [False]           # the unusable node does not count
    assert o["bind_create"] == [0] and o["bind_tenant_open"] is True
    assert o["bind_tenant_stat"] == "character special file 1:3 666 0"   # root-owned inside
    assert o["bind_invisible_here"] and o["bind_present"] == [True]
    assert o["bind_create_again"] == [1] and o["bind_second_node"] == [0]
    assert o["bind_remove"] == [0, 0] and o["after_remove_stat"] == ""
    assert o["after_remove_present"] == [False] and o["remove_again"] == [1]
    assert o["plain_remove_of_bound"] == [0] and o["plain_after"] == ""
