"""The plugin-lifetime contract at the C ABI from a C++ caller:
tests/plugin_lifetime.cpp, built with AddressSanitizer on its host code by tests/Makefile
(__graft_entry__.build()).  A plugin fails on its 500th hook call; the batch fails with
IPXG_EPLUGIN, the engine refuses work with IPXG_ESTATE; ipxg_destroy then calls nothing of the
failed plugin but free_ctx, once per copy it made; only then does the caller free its own
instance.  ASan reports a hook or free_ctx reaching freed memory, or a copy freed twice."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "plugin_lifetime")
# (the harness may preload a library of its own: ASan need not come first; HIP's own allocations
# are not this test's leaks)
ENV = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=0:abort_on_error=0")


def _run():
    assert os.path.exists(BIN), "tests/plugin_lifetime not built (make -C tests)"
    return subprocess.run([BIN], env=ENV, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)


def test_plugin_lifetime_program_without_gpu():
    """Without a GPU the program stops at ipxg_create (77), with its own instance released."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the gpu test runs the whole contract")
    r = _run()
    assert r.returncode == 77, r.stdout


@pytest.mark.gpu
def test_plugin_lifetime_contract():
    r = _run()
    assert r.returncode == 0 and "AddressSanitizer" not in r.stdout, r.stdout
    assert r.stdout.startswith("ok:"), r.stdout
