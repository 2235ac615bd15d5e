"""The failing fp32 train-step tests with a recorder around train._encoded: each batch's condition c as the step
starts (at yield) and as the step has been fully enqueued (before the generator resumes), vs the eager encoder."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import train as T_  # noqa: E402
import test_gpu_models as TM  # noqa: E402

dev = torch.device("cuda:0")
orig = T_._encoded
log = []


def rec(encoder, loader, device, optimizer):
    loader = list(loader)
    snaps = []
    stages = []
    for i, (c, m, x0) in enumerate(orig(encoder, loader, device, optimizer)):
        a = c.float().clone()
        ge = T_._ENC_GRAPHS[encoder]
        (slots,) = ge.cache.values()
        sl = slots[i % 2]
        stages.append((sl.inp.clone(), sl.h0.float().clone(), sl.h1.float().clone()))
        bb_ = encoder.backbone
        if os.environ.get("GC3_VERBOSE"):
            print("batch", i, "prep key", bb_._prep_key, "id", id(bb_._prep), "versions",
              [p_._version for p_ in bb_._plist][:8], "tables", [(k[:2], id(v[1])) for k, v in
                                                                 __import__("fddm_hip.runtime").runtime._tables.items()],
                  flush=True)
        yield c, m, x0
        snaps.append((a, c.float().clone()))
    torch.cuda.synchronize()
    refs = [encoder(w.to(device))[0].float().clone() for w, _ in loader]   # eager, after the epoch
    bb = encoder.backbone
    for i, (a, b) in enumerate(snaps):
        w = loader[i][0].to(device).float()
        h0 = bb.stage_conv0(w)
        h1 = bb.stage_conv1(h0)
        inp, g0, g1 = stages[i]
        log.append((i, float((a - refs[i]).abs().max()), float((b - refs[i]).abs().max()),
                    "inp", float((inp - w).abs().max()), "h0", float((g0 - h0.float()).abs().max()),
                    "h1", float((g1 - h1.float()).abs().max())))


class MP:
    def setattr(self, obj, name, val):
        setattr(obj, name, val)


T_._encoded = rec
for tag, geom, V, d, H, NL, FF, Tn in (("step_repeat", TM.SMALL_WAVLM, 500, 128, 2, 1, 256, 20),
                                        ("step_c1", {}, 8000, 128, 2, 2, 2048, 10),
                                        ("step_repeat", TM.SMALL_WAVLM, 500, 128, 2, 1, 256, 20)):
    if len(sys.argv) > 1 and tag not in sys.argv[1:]:
        continue
    log.clear()
    try:
        TM.test_train_step_fp32_matches_reference(tag, geom, V, d, H, NL, FF, Tn, MP())
        res = "pass"
    except AssertionError as e:
        res = "FAIL " + str(e)[:100]
    print(tag, res, "| c err (batch, at yield, after step):", log, flush=True)
