#!/usr/bin/env python3
"""Repeat the train -> checkpoint -> predict path of
tests/test_entrypoints.py::test_train_checkpoint_predict[raw] and report the
first non-finite tensor (loss history, parameters / BN buffers after
training, the predicted window probabilities), to chase a run-to-run NaN.
usage: python tools/ep_probe.py [repeats]"""
import json
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    raw = "--spec" not in sys.argv
    import audiomodel
    import build
    import predict
    from scipy.io import wavfile

    for it in range(reps):
        tmp = Path(tempfile.mkdtemp())
        assert build.main([str(tmp / "ds"), "--synthetic", "16", "--labels", "bird,noise", "--shards", "2"]) == 0
        td = tmp / "ds" / "training-data"
        args = audiomodel.parse_args(["run1", "-d", str(td), "--epochs", "1", "--batch-size", "4", "--model-name",
                                      "wr-resnet-bird", "--n_mels", "128", "--checkpoint-dir", str(tmp / "ck")]
                                     + (["--load-raw"] if raw else []))
        hist = audiomodel.train_model(args)
        ck = tmp / "ck" / "run1"
        sd = torch.load(ck / "model.pt", map_location="cpu", weights_only=True)
        bad = [k for k, v in sd.items() if torch.is_tensor(v) and v.is_floating_point() and not torch.isfinite(v).all()]
        rng = np.random.default_rng(3)
        rec = np.concatenate([build.synth_clip(rng, False) for _ in range(3)] + [build.synth_clip(rng, True)[:48000]])
        wavfile.write(tmp / "rec.wav", 48000, (rec * 32767).astype(np.int16))
        p = predict.Predictor(ck)
        r = p.predict_file(tmp / "rec.wav", stride=1.0, batch_size=4)
        wins = np.stack([rec[k * 48000:(k + 3) * 48000] for k in range(8)])
        a = p.predict_clips(wins, batch_size=8)
        # the eval forward's intermediates on the same windows
        from acfe import ops
        with torch.no_grad():
            x = torch.from_numpy(np.ascontiguousarray(wins, np.float32)).to(p.device)
            feats = p.frontend(x, pad_mode="constant")
            hm = p.model.head_maps(feats).float()
            l1 = ops.logmeanexp(hm, axis=1, sharpness=5).float()
            l2 = ops.logmeanexp(l1, axis=2, sharpness=5).float()
            z = p.model.prediction(l2).float()

        def st(t):
            f = torch.isfinite(t)
            return {"absmax_finite": float(t[f].abs().max()) if f.any() else None, "nan": int(torch.isnan(t).sum()),
                    "inf": int(torch.isinf(t).sum()), "n": t.numel()}
        inter = {"feats": st(feats.float()), "head": st(hm), "lme1": st(l1), "lme2": st(l2), "logits": st(z)}
        print(json.dumps({"it": it, "inter": inter, "loss": hist["loss"], "val_loss": hist["val_loss"], "bad_state": bad[:12],
                          "n_bad_state": len(bad), "mean": r["mean"], "clip_probs_finite": bool(np.isfinite(a).all()),
                          "lr": hist.get("learning_rate")}), flush=True)
        if bad:
            for k in bad[:6]:
                v = sd[k]
                print("   ", k, tuple(v.shape), "nan", int(torch.isnan(v).sum()), "inf", int(torch.isinf(v).sum()))


if __name__ == "__main__":
    main()
