"""Host code under AddressSanitizer+UBSan and ThreadSanitizer: matrix demo, SpMV, histogram
(pthreads barrier, OpenMP), and the native distributed region growing over the TCP transport with 4 ranks."""
import pytest

from parallel_c_programs_amd import sanitize


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_code_sanitizer_clean(tmp_path, kind):
    fails = sanitize.run_checks(kind, tmp_path)
    assert not fails, "\n".join(fails)
