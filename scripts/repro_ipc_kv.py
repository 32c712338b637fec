"""Debug helper for the KV IPC landing zone: decode worker subprocess + in-process IPCSender, step by step."""
import asyncio
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
fd, pf = tempfile.mkstemp()
os.close(fd)
os.unlink(pf)
log = open(os.path.join(ROOT, "gpurun_out", "repro_kv_worker.log"), "w")
cmd = [sys.executable, "-u", "-m", "src.worker", "--worker-id", "dec", "--host", "127.0.0.1", "--port", "0", "--port-file",
       pf, "--model", "mini", "--arch", "llama", "--preset", "llama-mini", "--role", "decode", "--max-batch-size", "8",
       "--max-model-len", "1024", "--num-kv-blocks", "256"]
p = subprocess.Popen(cmd, cwd=ROOT, stdout=log, stderr=log, env=dict(os.environ, DIE_DEBUG_IPC="1"))
t0 = time.time()
while not os.path.exists(pf) and time.time() - t0 < 200 and p.poll() is None:
    time.sleep(0.2)
port = int(open(pf).read())
print("worker up", port, round(time.time() - t0, 1), flush=True)


async def main():
    import torch
    from src.client import InferenceClient
    from src.parallel.kv_transfer import IPCSender

    c = InferenceClient(f"127.0.0.1:{port}", timeout=20)
    rep = await c.call({"op": "kv_channel", "model": "mini"})
    print("kv_channel", {k: v for k, v in rep.items() if k != "handle"}, flush=True)
    torch.zeros(1, device="cuda:0")
    print("opening", flush=True); t_open = time.time()
    s = IPCSender(rep.get("handles") or rep["handle"], rep.get("seg_bytes", rep["capacity"]), torch.device("cuda:0"))
    print("opened", [hex(p) for p in s.ptrs], round(time.time() - t_open, 2), "s", flush=True)
    r = await c.call({"op": "kv_reserve", "model": "mini", "nbytes": 1 << 20})
    print("reserve", r, flush=True)
    x = torch.arange(1 << 19, device="cuda:0", dtype=torch.int16).view(torch.bfloat16)
    s.write(r["offset"], x)
    print("written", flush=True)
    c.close()


try:
    asyncio.run(asyncio.wait_for(main(), 60))
finally:
    p.terminate()
    p.wait(30)
