"""The host parsers and packer under AddressSanitizer + UBSan:
tests/sanitize/run.py builds them host-only with -fsanitize=address,undefined
and drives every host entry point over the fixtures, the generated parity
cases and seeded mutations; any finding aborts the driver."""
import os
import shutil
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, 'sanitize'))


@pytest.mark.skipif(not os.path.exists('/opt/rocm/bin/hipcc') or shutil.which('nm') is None,
                    reason='needs hipcc')
def test_host_code_clean_under_asan_ubsan(capsys):
    import run
    rc = run.main(['--mutations', '5'])
    out = capsys.readouterr().out
    assert rc == 0, out[-4000:]
    assert '0 check failure(s)' in out
    assert 'ERROR: AddressSanitizer' not in out and 'runtime error' not in out
