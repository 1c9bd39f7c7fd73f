"""CPU timing of the native request codec (acs_codec_encode) on synthetic JSON requests.

usage: python tools/codec_prof.py [c3|c2] [requests] [threads] [reps] [second_role]
Prints per-rep seconds of parse+encode / regex / classes / total and requests/s.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
from acs_mi355x import compiler, store, synth  # noqa: E402
from acs_mi355x.codec import NativeCodec  # noqa: E402
from acs_mi355x.config import SERVICE_URNS, COMBINING_ALGORITHMS  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    second = float(sys.argv[5]) if len(sys.argv) > 5 else 0.5
    doc = synth.c2_store() if kind == "c2" else synth.c3_store()
    cs = compiler.compile_store(store.populate(doc), SERVICE_URNS, COMBINING_ALGORITHMS)
    sb = synth.requests(cs, n, kind, seed=0xACC1000, second_role=second if kind != "c2" else 0.0)
    idx = np.arange(n)
    t0 = time.perf_counter()
    text = sb.json_text(idx)
    print(f"json: {len(text) / n:.0f} B/request, generated in {time.perf_counter() - t0:.1f}s", flush=True)
    codec = NativeCodec(compiler.store_blob(cs))
    if kind != "c2":
        for k, v in sb.hrs_forests(idx).items():
            codec.set_subject_scopes(k, v)
    for r in range(reps):
        t0 = time.perf_counter()
        b = codec.encode(text, threads=threads)
        dt = time.perf_counter() - t0
        st = b.stats()
        print(f"rep {r}: {dt:.3f}s  {n / dt / 1e6:.3f} M req/s  encode {st['encode_s']:.3f} regex {st['regex_s']:.3f} "
              f"classes {st['classes_s']:.3f} total {st['total_s']:.3f}  classes={b.cand.shape[0]}", flush=True)
        b.close()
    codec.close()


if __name__ == "__main__":
    main()
