#!/usr/bin/env python3
"""Interactive KV cache CLI (commands as in the reference's kvstore demo):
get/set/delete/batch_get/batch_set/list/clear/stats/ttl/save/help/exit.
Also `blocks` shows the paged KV-block manager (native) in action."""

import argparse
import json
import os
import shlex
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.kvstore import KVCache  # noqa: E402

HELP = """get K | set K V [ttl] | delete K | batch_get K1 K2 .. | batch_set K1=V1 K2=V2 ..
list | clear | stats | ttl K SECONDS | save [path] | blocks | help | exit"""


def blocks_demo():
    from src.engine.block_manager import KVBlockManager
    from src.engine.sequence import Sequence
    from src.preproc import SamplingParams

    bm = KVBlockManager(num_blocks=8, block_size=4)
    a = Sequence("a", list(range(17)), SamplingParams())
    bm.allocate(a)
    a.num_computed = 17  # pretend the prefill ran
    bm.register_prompt_blocks(a)
    print("seq a blocks", a.block_table, bm.stats())
    bm.free(a)
    b = Sequence("b", list(range(17)) + [99], SamplingParams())
    bm.allocate(b)
    print("seq b reuses prefix blocks", b.block_table, "prefix hit tokens", b.num_prefix_hit)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-size", type=int, default=100)
    ap.add_argument("--policy", default="lru", choices=["lru", "lfu", "fifo"])
    ap.add_argument("--ttl", type=float, default=None)
    ap.add_argument("--persist", default=None)
    a = ap.parse_args()
    kv = KVCache(a.max_size, a.policy, a.ttl, persist_path=a.persist)
    print(HELP)
    while True:
        try:
            line = input("kv> ").strip()
        except EOFError:
            break
        if not line:
            continue
        cmd, *args = shlex.split(line)
        try:
            if cmd == "exit":
                break
            elif cmd == "help":
                print(HELP)
            elif cmd == "get":
                print(kv.get(args[0]))
            elif cmd == "set":
                kv.set(args[0], args[1], ttl=float(args[2]) if len(args) > 2 else None)
            elif cmd == "delete":
                print(kv.delete(args[0]))
            elif cmd == "batch_get":
                print(kv.batch_get(args))
            elif cmd == "batch_set":
                kv.batch_set(dict(x.split("=", 1) for x in args))
            elif cmd == "list":
                print(list(kv.cache.keys()))
            elif cmd == "clear":
                kv.clear()
            elif cmd == "stats":
                print(json.dumps(kv.get_stats(), indent=2))
            elif cmd == "ttl":
                v = kv.get(args[0])
                kv.set(args[0], v, ttl=float(args[1]))
            elif cmd == "save":
                print(kv.save(args[0] if args else None))
            elif cmd == "blocks":
                blocks_demo()
            else:
                print("unknown command;", HELP)
        except (IndexError, ValueError) as e:
            print("error:", e)
    kv.close()


if __name__ == "__main__":
    main()
