"""Worker process lifecycle on CPU: SIGTERM / SIGINT end the serve loop cleanly (exit 0, no asyncio
"Task exception was never retrieved" noise — round 3's worker raised SystemExit inside a task), as the
reference's signal handlers promise (`/root/reference/src/worker.py:43-49,63-82`)."""

import os
import signal
import subprocess
import sys
import tempfile
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("sig", [signal.SIGTERM, signal.SIGINT])
def test_worker_signal_shutdown_is_clean(sig):
    fd, pf = tempfile.mkstemp()
    os.close(fd)
    os.unlink(pf)
    p = subprocess.Popen([sys.executable, "-m", "src.worker", "--worker-id", "sig", "--host", "127.0.0.1",
                          "--port", "0", "--port-file", pf, "--mock-latency-ms", "1"],
                         cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        t0 = time.time()
        while not os.path.exists(pf):
            assert p.poll() is None, p.communicate()
            assert time.time() - t0 < 60
            time.sleep(0.05)
        p.send_signal(sig)
        out, err = p.communicate(timeout=30)
    finally:
        if p.poll() is None:
            p.kill()
        if os.path.exists(pf):
            os.unlink(pf)
    assert p.returncode == 0, (p.returncode, err[-2000:])
    assert "never retrieved" not in err and "Traceback" not in err, err[-2000:]
    assert "shutting down" in err
