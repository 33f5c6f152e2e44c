"""Turn a tools/pmc_summary.py summary into profiles/layer_traffic.json (read by bench.py as
roofline.traffic): HBM-side bytes per residual-layer launch = FETCH_SIZE*1024*2 (gfx950 reports
half the bytes of wide coalesced reads, MI355X_MICROARCH.md sec HBM) + WRITE_SIZE*1024, averaged
over the middle-layer launches of the profiled bench run."""
import json
import sys


def main(summary, out, config="libritts_v1", utts=32, layer_kernel="split"):
    d = json.load(open(summary))
    if layer_kernel.startswith("split"):
        # middle layers: not last, and not layer 0 with the fused first_conv (<false, TC, true>)
        rows = {k: v for k, v in d.items() if ("layer_%s_kernel<false" % layer_kernel) in k and ", true>" not in k}
    else:
        rows = {k: v for k, v in d.items() if "layer" in k and ("0, 16" in k or "4, 4, 0" in k)}
    k, v = max(rows.items(), key=lambda kv: kv[1].get("SQ_WAVES", 0))
    res = {
        "config": config,
        "utts": utts,
        "layer_kernel": layer_kernel,
        "kernel": k,
        "fetch_bytes_per_launch": v["FETCH_BYTES_corrected"],
        "write_bytes_per_launch": v["WRITE_BYTES"],
        "hbm_bytes_per_launch": v["FETCH_BYTES_corrected"] + v["WRITE_BYTES"],
        "mfma_insts_per_launch": v["SQ_INSTS_MFMA"],
        "mfma_busy": v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] / 8 * 1024),
        "l2_hit": v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]),
        "source": summary,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], layer_kernel=sys.argv[3] if len(sys.argv) > 3 else "split")
