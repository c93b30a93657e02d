"""Debug helper: reproduce the first failing ShortWritings block of a hint
alone at the same 1 KiB alignment, with kernel printf (VSA_DEBUG_FLAGS=4)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import vectorscan_amd as vsa, oracle
from test_gpu_parity import batch_run
from test_cpu_oracle import load, build_or_none
ctx = vsa.Context(0)
spec = load("fdr_shortwritings.json")[0]
bufs = [bytes.fromhex(x) for x in spec["bufs"]]
pats = [bytes.fromhex(x) for x in spec["pats"]]
hint = int(sys.argv[1]) if len(sys.argv) > 1 else 9
found = None
for g in range(0, len(pats), 32):
    lits = [vsa.HwlmLiteral(p, False, g + i) for i, p in enumerate(pats[g:g + 32])]
    blob = build_or_none(lits, hint)
    if blob is None:
        continue
    got = batch_run(ctx, blob, bufs)
    for bi, (b, m) in enumerate(zip(bufs, got)):
        st, mo = oracle.fdr_exec(vsa.engine_blob(blob), b)
        if m != mo:
            found = (g, bi, blob)
            break
    if found:
        break
g, bi, blob = found
off = sum(len(b) + 3 for b in bufs[:bi])
b = bufs[bi]
print("group", g, "block", bi, "off", off, "mod1024", off % 1024, "len", len(b), "data", b.hex())
for mis in (off % 1024, off % 1024 + 1024, off % 16):
    if mis in (off % 1024, off % 16):
        os.environ["VSA_DEBUG_FLAGS"] = "4"
    got = batch_run(ctx, blob, [b], misalign=mis)[0]
    os.environ.pop("VSA_DEBUG_FLAGS", None)
    st, mo = oracle.fdr_exec(vsa.engine_blob(blob), b)
    print("mis", mis, "ok" if got == mo else "BAD", "\n gpu", got, "\n orc", mo, flush=True)
# also: the full batch restricted to blocks bi-1..bi
got = batch_run(ctx, blob, bufs[:bi + 1])
st, mo = oracle.fdr_exec(vsa.engine_blob(blob), b)
print("prefix batch", "ok" if got[bi] == mo else "BAD", flush=True)
