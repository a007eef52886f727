"""Debug aid for the plugin pre-classification inside k_bin (Params::plug): the fuzz corpus of
tests/test_plugins.py::test_classifier_payload_offsets_on_fuzz_corpus through the engine with the
fold and with the separate k_classify pass (IPXG_CLASSIFY_PASS=1); for the flows whose extension
bit differs, the packets' shapes (caplen, alignment, parse fields, payload bytes).

  python3 tools/dbg_fold.py [batch]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(batch):
    import numpy as np
    import synth
    import test_plugins
    from ipfixprobe_amd import Engine, run_capture
    arena, desc = synth.to_batch(synth.fuzz_corpus(20000, seed=71))
    res = {}
    for mode in ("fold", "pass"):
        if mode == "pass":
            os.environ["IPXG_CLASSIFY_PASS"] = "1"
        else:
            os.environ.pop("IPXG_CLASSIFY_PASS", None)
        pl = test_plugins.PrefixMarker()
        got, st = run_capture(arena, desc, params="s=18", batch=batch, plugins=[pl.struct])
        res[mode] = {int(r["flow_hash"]): int(r["ext"]) for r in got}
        print(mode, "hooks saw rule packets:", pl.seen, {k: st[k] for k in ("complex_flows", "walked_packets",
                                                                           "new_keys" if "new_keys" in st else "batches")})
    diff = sorted(h for h in res["pass"] if res["pass"][h] != res["fold"].get(h))
    print("flows with a different ext: %d (fold ext=1: %d, pass ext=1: %d)" % (
        len(diff), sum(1 for h in diff if res["fold"].get(h)), sum(1 for h in diff if res["pass"][h])))
    with Engine("s=18") as e:
        pk = e.parse(arena, desc)
    d = desc.view(np.uint32).reshape(-1, 4)
    want = set(diff)
    shown = 0
    for i in range(len(pk)):
        h = int(pk["hash_fwd"][i])
        if h not in want and int(pk["hash_inv"][i]) not in want:
            continue
        off, cl = int(d[i, 0]), int(d[i, 1]) & 0xFFFF
        po, pln = int(pk["payload_off"][i]), int(pk["payload_len"][i])
        pay = bytes(arena[off + po: off + min(po + 4, cl)]) if po < cl else b""
        print("pkt %6d caplen %4d off%%16 %2d ether %04x ipv %d proto %3d l4 ports %5d %5d frag %d ip_len %4d "
              "payload_off %3d len %4d bytes %s" % (
                  i, cl, off % 16, int(pk["ethertype"][i]), int(pk["ip_version"][i]), int(pk["ip_proto"][i]),
                  int(pk["src_port"][i]), int(pk["dst_port"][i]), int(pk["frag_off"][i]), int(pk["ip_len"][i]),
                  po, pln, pay.hex()))
        shown += 1
        if shown >= 60:
            break


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else None)
