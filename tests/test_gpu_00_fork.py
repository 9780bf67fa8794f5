"""Fork safety of the drop-in (GPU).  Named to run FIRST in the GPU session:
main.py's parent never starts HIP before it forks, and neither may this
process before fork_dropin.run() (it checks).  See tests/fork_dropin.py."""
import pytest

import fork_dropin
from ldpc_amd import _lib


@pytest.mark.gpu
def test_main_py_threads_pattern_bit_exact():
    """Parent builds SPA_Decoder (main.py:221), 2 forked workers build their own
    and decode the reference's golden frames (main.py:78, :248-256): bit-exact."""
    if _lib.hip_started_here():
        pytest.fail("HIP already started in this process: run this file first (or tests/fork_dropin.py "
                    "as a script)")
    bad, pids = fork_dropin.run(workers=2, frames=16)
    assert bad == [], f"frames differing from the reference: {bad}"
    assert len(pids) >= 1


@pytest.mark.gpu
def test_child_forked_after_hip_refuses():
    """A child forked after its parent started HIP gets LdpcError, not a hang."""
    assert fork_dropin.run_poisoned() == "refused"
