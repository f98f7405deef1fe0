#!/usr/bin/env python
"""Benchmark: Mask R-CNN R50-FPN at 1333x800 on MI355X (img/s).

Default (--mode train, BASELINE.json config C3 / the north_star target): one
step = one data-parallel training iteration at 2 images per GPU — forward,
RPN / Fast R-CNN / mask losses, backward with the bucketed RCCL gradient
all-reduce overlapped, per-tensor clip and the Momentum-SGD update — over
synthetic COCO-shaped images + GT already resident in HBM.  value = all
ranks' images / (max-over-ranks time of K steps), weak scaling.

--mode infer: one step = one batched forward of the whole model over
synthetic images already resident in HBM: ResNet-50 (every conv but the frozen
7x7 stem on the HIP split-product MFMA kernels, FrozenBN folded) -> FPN (MFMA
kernels, fused top-down add) -> RPN head (MFMA) + fused top-k/decode/NMS
proposals -> multi-level ROIAlign 7x7 -> box head (fc1 on the MFMA kernel,
fc2 / predictors hipBLASLt) -> fused
Fast R-CNN post-processing (softmax/decode/clip/class-offset NMS) -> ROIAlign
14x14 on the detections -> mask head (MFMA) -> per-class mask sigmoid.

Weights are random-init with the reference initialisers; as BASELINE.md
prescribes, the class / objectness logit scales are calibrated once
(box-head class logits ~ N(0, 3^2), RPN objectness ~ N(0, 1)) so that the
score thresholds and NMS see realistic survivor counts (reported).

Multi-GPU: one process per GPU (torchrun), each rank runs its own images
(inference: "replicas", no data-path collective; training: DP with one
gradient all-reduce per step), barrier +
synchronize around the timed region, time = max over ranks, value = all
images / that time (weak scaling).
"""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    "mask_rcnn_R_50_FPN": "configs/COCO-InstanceSegmentation/mask_rcnn_R_50_FPN_1x.yaml",
    "faster_rcnn_R_50_FPN": "configs/COCO-Detection/faster_rcnn_R_50_FPN_1x.yaml",
    "retinanet_R_50_FPN": "configs/COCO-Detection/retinanet_R_50_FPN_1x.yaml",
    "retinanet_R_101_FPN": "configs/COCO-Detection/retinanet_R_101_FPN_3x.yaml",
    "solo_v2_R_50_FPN": "configs/COCO-InstanceSegmentation/solo_v2_R_50_FPN_1x.yaml",
}
METRICS = {
    "mask_rcnn_R_50_FPN": "img/sec whole-node Mask R-CNN R50-FPN @1333x800",
    "faster_rcnn_R_50_FPN": "img/sec Faster R-CNN R50-FPN @1333x800",
    "retinanet_R_50_FPN": "img/sec RetinaNet R50-FPN",
    "retinanet_R_101_FPN": "img/sec RetinaNet R101-FPN dense anchors",
    "solo_v2_R_50_FPN": "img/sec SOLOv2 R50-FPN (dynamic-conv masks + Matrix NMS)",
}
MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32)
# split products: every f32 multiply-add costs six v_mfma_f32_32x32x16_bf16
# products, so the f32-equivalent ceiling is the dense BF16 MFMA peak / 6
# (MI355X_MICROARCH.md: ~2.5 PF dense BF16)
MFMA_SPLIT_PEAK_TFLOPS = round(2500.0 / 6, 1)
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s
# MI355X_MICROARCH.md: I8 MFMA (32x32x32) at 2x the BF16 rate per clock
MFMA_I8_PEAK_TOPS = 2 * 2500.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # (30: the one eager step that carries the per-launch HIP events -- the
    # live roofline -- is one of the timed steps; among 10 it weighed ~1 % of
    # the line, among 30 a third of that; 30 steps still take < 1 s)
    # (60: the one event-timed sample step -- eager, HIP events around every
    # hot launch, ~6 ms more than a replay -- is 1/60 of the timed region;
    # at 30 steps it cost the line 1.1 %, profiles/r6aw_sample_step_cost.txt)
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=2, help="images per GPU per step")
    p.add_argument("--model", default="mask_rcnn_R_50_FPN", choices=sorted(CONFIGS))
    p.add_argument("--height", type=int, default=800)
    p.add_argument("--width", type=int, default=1333)
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle (rank 0, N=1)")
    p.add_argument("--cpu-images", type=int, default=2, help="images per CPU iteration (<= batch)")
    p.add_argument("--cpu-iters", type=int, default=5,
                   help="timed CPU iterations (median).  BASELINE.md section 2 asks 3 warm-ups + "
                        "the median of 20 per OP (cpu_per_op_c2 does that); a whole training "
                        "iteration takes ~4 s on 16 threads, so the step-level sample is bounded "
                        "to 1 warm-up + the median of 5 (~25 s, the CPU-sample budget)")
    p.add_argument("--cpu-one-core", type=int, default=1, help="also time 1 image on 1 core")
    p.add_argument("--no-kernel-timing", action="store_true")
    p.add_argument("--no-calibration", action="store_true",
                   help="skip the box calibration GEMM / conv before the timed region")
    p.add_argument("--timed-step-sample", type=int, default=-1,
                   help="timed step whose kernel launches carry HIP events (-1: the last)")
    p.add_argument("--mode", default="train", choices=["train", "infer"])
    p.add_argument("--mask-format", default="conventional", choices=["conventional", "raw", "fixed"],
                   help="inference mask output (SEGMENTATION_OUTPUT.FORMAT)")
    p.add_argument("--bucket-mb", type=int, default=32, help="all-reduce bucket size (train)")
    p.add_argument("--graphs", type=int, default=1,
                   help="train: replay the step from hipGraphs (engine/graphed.py; at world "
                        "size > 1 the all-reduces run between the backward and update graphs); "
                        "0 = the eager Trainer.step")
    p.add_argument("--wgrad-side", type=int, default=0,
                   help="train, graphed: the convs' weight gradients captured on a side stream "
                        "beside their data gradients (1) or on the step's one stream (0)")
    p.add_argument("--fixed-rows-steps", type=int, default=10,
                   help="train (default run): after the main timed region, also time this many "
                        "steps with the fixed 256-row mask branch (a second object in the "
                        "line); 0 = skip")
    p.add_argument("--mask-fixed-rows", action="store_true",
                   help="train: the mask head on the fixed BATCH_SIZE_PER_IMAGE x "
                        "POSITIVE_FRACTION rows per image (128 at the defaults, "
                        "defaults.py:413-415; the steady-state load of a trained model) "
                        "instead of the step's foreground rows")
    return p.parse_args()


def build(args, device):
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    from detectron2_tensorflow_amd.modeling import build_model
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, CONFIGS[args.model]))
    # inference: the reference's default output format (masks pasted onto the
    # padded canvas as uint8, detector_postprocess); training never pastes
    cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT = args.mask_format if args.mode == "infer" else "raw"
    cfg.SOLVER.IMS_PER_GPU = args.batch
    finalize(cfg, training=args.mode == "train", world_size=args.gpus,
             category_map={"num_thing_classes": 80, "num_stuff_classes": 53,
                           "stuff_ignore_value": 0})
    torch.manual_seed(0)
    model = build_model(cfg).to(device)
    model.train(args.mode == "train")
    return cfg, model


def is_single_stage(model):
    return hasattr(model, "detector")


@torch.no_grad()
def calibrate_retinanet(model, batch):
    """BASELINE.md injection for RetinaNet: class logits ~ N(-3, 1), deltas ~
    N(0, 0.1^2) on this batch's features (utils/synthetic.py)."""
    from detectron2_tensorflow_amd.utils.synthetic import calibrate_retinanet_head
    det = model.detector
    feats = model.neck(model.backbone(model.preprocess_image(batch).tensor))
    cls, box = det.head([feats[f] for f in det.in_features])
    calibrate_retinanet_head(det.head, cls, box)


@torch.no_grad()
def calibrate_solo(model, batch):
    """Score injection for SOLOv2: category logits ~ N(-4.5, 1) (a few hundred
    to a few thousand candidates above 0.1 after point NMS), dynamic kernels
    of std 0.1 (utils/synthetic.py)."""
    from detectron2_tensorflow_amd.utils.synthetic import calibrate_solo_head
    b = model.detector.mask_kernel_branch
    feats = model.neck(model.backbone(model.preprocess_image(batch).tensor))
    cls, ker = b(feats)
    calibrate_solo_head(b, cls, ker)


def is_solo(model):
    return hasattr(getattr(model, "detector", None), "mask_kernel_branch")


@torch.no_grad()
def calibrate_scores(model, batch):
    """Rescale the class / objectness logit weights so the random-init model
    emits BASELINE.md's synthetic score distributions, and the RPN anchor
    deltas to N(0, 0.1^2): the unnormalised features of a random-init ResNet
    otherwise give deltas of O(10), which collapse most proposals onto the
    image border (a random-init artefact, not a training distribution)."""
    if is_solo(model):
        return calibrate_solo(model, batch)
    if is_single_stage(model):
        return calibrate_retinanet(model, batch)
    from detectron2_tensorflow_amd.utils.synthetic import calibrate_rcnn_scores
    calibrate_rcnn_scores(model, batch)


def synthetic_batch(args, device, rank):
    from detectron2_tensorflow_amd.utils.synthetic import synthetic_images, synthetic_train_batch
    if args.mode == "train":
        # SOLOv2 takes its GT masks at the padded image size (solo_v2.py:399-401)
        full = ((-(-args.height // 32) * 32, -(-args.width // 32) * 32)
                if args.model.startswith("solo") else None)
        return synthetic_train_batch(args.batch, args.height, args.width, 1000 + rank, device,
                                     full_mask_hw=full)
    return synthetic_images(args.batch, args.height, args.width, 1000 + rank, device)


def _latest_pmc():
    """The newest round's committed PMC summary (profiles/rNN_train_pmc.json)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_train_pmc.json")))
    return files[-1] if files else os.path.join(ROOT, "profiles", "r1_train_pmc.json")


PMC_FILE = _latest_pmc()
# ``traffic`` is NOT measured by this run: it is the builder's committed
# rocprofv3 PMC bytes per launch (same bench command, builder's box); the
# ``achieved_counter`` / ``frac_counter`` figures divide those bytes by THIS
# run's kernel times
TRAFFIC_SOURCE = ("builder-committed rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE per launch), "
                  + os.path.relpath(PMC_FILE, ROOT))


# kernels whose PMC-counted bytes belong to the default (foreground-row)
# training workload only: --mask-fixed-rows changes their work
PMC_SKIP = set()
# groups whose PMC "launch" is one op call made of several HIP-event launches
# (tools/pmc_summarize.py: the ROIAlign backward's main kernel is its one
# roi_bwd_clear per backward): op calls per training step
PMC_OPS_PER_STEP = {"roi_align_bwd": 1}


def pmc_traffic(group, mode):
    """HBM bytes per launch of a kernel group from the committed rocprofv3 PMC
    passes (tools/pmc_traffic.sh: FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected)
    of this same bench command in training mode; None when not available."""
    if mode != "train" or not os.path.exists(PMC_FILE) or group in PMC_SKIP:
        return None
    try:
        with open(PMC_FILE) as f:
            g = json.load(f)["groups"].get(group)
        return round(g["traffic_bytes_per_launch"]) if g else None
    except (OSError, ValueError, KeyError):
        return None


def kernel_report(summary, mode="infer", extras=None):
    """Roofline objects from the live HIP-event timings of the timed region.
    Convs are reported per product form: "conv2d_split" (f32 operands split
    into 3 bf16 terms, 6 bf16 MFMA products; peak = BF16 dense / 6) and
    "conv2d_mfma" (f32 MFMA products; peak = FP32 matrix).

    HBM-bound kernels: ``achieved`` / ``frac`` use the launch's UNIQUE bytes
    where a model exists (ROIAlign: the distinct feature rows the samples
    read + the output written, forward; grad_out read + the dense gradient
    maps written, backward) -- the least traffic that can serve the launch,
    so frac <= 1 -- with the SURVEY 8d D4 figure (4 corner reads per sample,
    which neighbouring bins share in cache) beside it as ``achieved_d4`` and
    the rocprofv3 PMC bytes of the same kernel (``traffic``, training only)
    as ``achieved_counter`` / ``frac_counter``."""
    extras = extras or {}
    rep = {}
    convs = (("conv2d_split", MFMA_SPLIT_PEAK_TFLOPS, "conv2d_split"),
             ("conv2d_mfma", MFMA_F32_PEAK_TFLOPS, "conv2d_mfma"),
             ("conv2d_wgrad_split", MFMA_SPLIT_PEAK_TFLOPS, "conv_wgrad_split"),
             ("conv2d_wgrad_mfma", MFMA_F32_PEAK_TFLOPS, "conv_wgrad"))
    for name, peak, pmc_group in convs:
        if name not in summary:
            continue
        n, ms, flops = summary[name]
        ach = flops / (ms * 1e-3) / 1e12
        rep[name] = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak,
                     "unit": "TFLOP/s", "frac": round(ach / peak, 4),
                     "traffic": pmc_traffic(pmc_group, mode), "traffic_source": TRAFFIC_SOURCE,
                     "launches": n,
                     "avg_us": round(ms * 1e3 / n, 2), "algorithmic_per_launch": flops / n}
    # the same conv launches split by their own bound (ops.bound_of: flop/B
    # against the product form's ridge): MFMA-bound shapes against the MFMA
    # peak, memory-bound shapes (the short-K residual 1x1s, ...) against HBM
    for base, peak in (("conv2d_split", MFMA_SPLIT_PEAK_TFLOPS),
                       ("conv2d_wgrad_split", MFMA_SPLIT_PEAK_TFLOPS),
                       ("conv2d_mfma", MFMA_F32_PEAK_TFLOPS)):
        for bound in ("mfma", "hbm"):
            name = f"{base}_{bound}_bound"
            if name not in summary:
                continue
            n, ms, flops = summary[name]
            sec = ms * 1e-3
            byts = extras.get(name, {}).get("bytes", 0.0)
            tf = flops / sec / 1e12
            gbs = byts / sec / 1e9
            r = {"bound": bound, "launches": n, "avg_us": round(ms * 1e3 / n, 2),
                 "ms_per_step": round(ms, 3), "achieved_tflops": round(tf, 2),
                 "achieved_gbs": round(gbs, 1), "flop_per_byte": round(flops / max(byts, 1.0), 1),
                 "bytes_model": "every operand read once + the output written once"}
            if bound == "mfma":
                r.update(achieved=round(tf, 2), peak=peak, unit="TFLOP/s", frac=round(tf / peak, 4))
            else:
                r.update(achieved=round(gbs, 1), peak=HBM_PEAK_GBPS, unit="GB/s",
                         frac=round(gbs / HBM_PEAK_GBPS, 4))
            rep[name] = r
    if "solo_matrix_nms" in summary:
        # int8 MFMA intersections (r6): 2 N^2 HW ops per image
        n, ms, ops_ = summary["solo_matrix_nms"]
        ach = ops_ / (ms * 1e-3) / 1e12
        rep["solo_matrix_nms"] = {"bound": "mfma", "achieved": round(ach, 1),
                                  "peak": MFMA_I8_PEAK_TOPS, "unit": "TOP/s",
                                  "frac": round(ach / MFMA_I8_PEAK_TOPS, 4),
                                  "ops_model": "2*k^2*Hm*Wm per image (SURVEY 8d D4)",
                                  "launches": n, "avg_us": round(ms * 1e3 / n, 2),
                                  "algorithmic_per_launch": ops_ / n}
    for name in ("roi_align_fwd", "roi_align_fwd_mask", "roi_align_bwd", "retinanet_postprocess",
                 "solo_mask_stats",
                 "solo_matrix_nms_popcount", "solo_paste"):
        if name not in summary:
            continue
        n, ms, byts = summary[name]
        sec = ms * 1e-3
        uniq = extras.get(name, {}).get("unique_bytes")
        model = uniq if uniq is not None else byts
        ach = model / sec / 1e9
        traffic = pmc_traffic(name, mode)
        r = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS,
             "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4),
             "bytes_model": "unique" if uniq is not None else "algorithmic",
             "traffic": traffic, "traffic_source": TRAFFIC_SOURCE if traffic else None,
             "launches": n, "avg_us": round(ms * 1e3 / n, 2),
             "algorithmic_per_launch": model / n}
        if uniq is not None:
            r["achieved_d4"] = round(byts / sec / 1e9, 1)
            r["d4_per_launch"] = byts / n
        if traffic:
            # the PMC group's "launch" is one op call: for the ROIAlign
            # backward that is the whole backward of the step (its phase-1
            # launch and the deferred per-level pixel passes, n HIP-event
            # launches together), so the counter bytes cover all n launches
            units = PMC_OPS_PER_STEP.get(name, n)
            if name in PMC_OPS_PER_STEP:
                r["traffic_per"] = "backward op (all of its launches in the step)"
            ac = traffic * units / sec / 1e9
            r["achieved_counter"] = round(ac, 1)
            r["frac_counter"] = round(ac / HBM_PEAK_GBPS, 4)
        rep[name] = r
    return rep


def box_calibration(device, iters=20):
    """Same-process calibration of THIS box, timed before the timed region so
    that a slow box can be told apart from a code regression:
    ``box_mfma_tflops`` = a fixed vendor bf16 GEMM (torch.matmul ->
    hipBLASLt, 8192^3, dense TF/s; the library is fixed by the image, so it
    moves only with the box's clocks / power), ``box_conv_p2_us`` = this
    repo's split-product conv on the FPN p2 3x3 shape (2x200x336x256 -> 256,
    the step's largest conv) in us per launch, with its f32-equivalent TF/s."""
    out = {}
    try:
        n = 8192
        a = torch.randn(n, n, device=device, dtype=torch.bfloat16)
        b = torch.randn(n, n, device=device, dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(a, b)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            torch.matmul(a, b)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / iters
        out["box_mfma_tflops"] = round(2.0 * n ** 3 / (ms * 1e-3) / 1e12, 1)
        out["box_mfma_gemm"] = f"bf16 torch.matmul {n}^3 (hipBLASLt), mean of {iters} launches"
        del a, b
        from detectron2_tensorflow_amd.layers import ops
        g = torch.Generator(device=device).manual_seed(0)
        x = torch.randn(2, 200, 336, 256, device=device, generator=g)
        w = torch.randn(3, 3, 256, 256, device=device, generator=g) * 0.02
        for _ in range(3):
            ops.conv2d_nhwc(x, w, None, 1, (1, 1))
        e0.record()
        for _ in range(iters):
            ops.conv2d_nhwc(x, w, None, 1, (1, 1))
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        out["box_conv_p2_us"] = round(us, 1)
        out["box_conv_p2_tflops"] = round(2.0 * 2 * 200 * 336 * 256 * 9 * 256 / (us * 1e-6) / 1e12, 1)
    except Exception as e:  # calibration is informative only
        out["box_calibration_error"] = f"{type(e).__name__}: {e}"
    return out


class GpuSampler:
    """Samples the GPU's gfx clock, memory clock, socket power and hotspot
    temperature (amdsmi gpu_metrics) every ``period`` s on a host thread while
    the timed region runs; summary() gives min / median / max of each.  If
    amdsmi is absent or refuses (a non-root user may not read every sensor)
    the line says so instead."""

    def __init__(self, device, period=0.05):
        import threading
        self.period = period
        self.samples = []
        self.error = None
        self._stop = threading.Event()
        self._thread = None
        self._h = None
        try:
            import amdsmi
            self._smi = amdsmi
            amdsmi.amdsmi_init()
            hs = amdsmi.amdsmi_get_processor_handles()
            props = torch.cuda.get_device_properties(device)
            want = (props.pci_domain_id, props.pci_bus_id, props.pci_device_id)
            for h in hs:
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
                dom, bus, rest = bdf.split(":")
                if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                    self._h = h
                    break
            if self._h is None:
                self.error = f"no amdsmi handle matches the device's PCI address {want}"
        except Exception as e:
            self.error = f"amdsmi unavailable: {type(e).__name__}: {e}"

    def _read(self):
        m = self._smi.amdsmi_get_gpu_metrics_info(self._h)

        def num(v):
            if isinstance(v, (list, tuple)):
                v = [x for x in v if isinstance(x, (int, float)) and x < 0xFFFF]
                return sum(v) / len(v) if v else None
            return v if isinstance(v, (int, float)) and v < 0xFFFF else None
        return {"gfxclk_mhz": num(m.get("current_gfxclks")) or num(m.get("current_gfxclk")),
                "uclk_mhz": num(m.get("current_uclk")),
                "power_w": num(m.get("current_socket_power")) or num(m.get("average_socket_power")),
                "hotspot_c": num(m.get("temperature_hotspot"))}

    def _run(self):
        while not self._stop.is_set():
            try:
                self.samples.append(self._read())
            except Exception as e:
                self.error = f"amdsmi read failed: {type(e).__name__}: {e}"
                return
            self._stop.wait(self.period)

    def start(self):
        if self._h is None:
            return
        import threading
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()

    def stop(self):
        if self._thread is not None:
            self._stop.set()
            self._thread.join()

    def summary(self):
        if not self.samples:
            return {"error": self.error or "no samples"}
        out = {"samples": len(self.samples), "period_s": self.period}
        for k in self.samples[0]:
            v = sorted(s[k] for s in self.samples if s.get(k) is not None)
            if v:
                out[k] = {"min": round(v[0], 1), "median": round(v[len(v) // 2], 1),
                          "max": round(v[-1], 1)}
        if self.error:
            out["error"] = self.error
        return out


def cpu_model_name():
    """The host CPU's model name (lscpu's "Model name", from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.lower().startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _median_time(fn, iters, warm=0):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], ts


def cpu_per_op_c2(batch, cores, reps=20):
    """the hot-path ops of the CPU
    restatement on one 1333x800 image (seeded synthetic inputs of the
    bench geometry), each 3 warm-ups + the median of ``reps`` runs, in ms:
    ROIAlign 7x7 over p2..p5 with 1,000 ROIs (SURVEY D2 boxes), the RPN
    proposals (anchors + decode + per-level top-k 1000 + NMS over 5 levels,
    post 1000), class-offset Fast R-CNN NMS (1,000 ROIs x 80 classes), and
    anchor generation + delta decode of all 268,569 anchors."""
    import numpy as np
    import oracle
    rng = np.random.default_rng(0)
    H, W, TH, TW = 800, 1344, 800, 1333
    strides = [4, 8, 16, 32]
    feats = [rng.normal(size=(1, H // s, W // s, 256)).astype(np.float32) for s in strides]
    c = rng.uniform([0, 0], [TH, TW], size=(1000, 2))
    sz = np.exp(rng.uniform(np.log(16), np.log(800), size=1000))
    ar = np.exp(rng.uniform(np.log(0.5), np.log(2.0), size=1000))
    h, w = sz * np.sqrt(ar), sz / np.sqrt(ar)
    boxes = np.stack([c[:, 0] - h / 2, c[:, 1] - w / 2, c[:, 0] + h / 2, c[:, 1] + w / 2],
                     1).astype(np.float32)
    bimg = np.zeros(1000, np.int32)
    out = {}
    t, _ = _median_time(lambda: oracle.roi_pooler(feats, boxes, bimg, (7, 7),
                                                  [1.0 / s for s in strides], 0, True), reps, 3)
    out["roi_align_7x7_1000rois_ms"] = round(t * 1e3, 3)
    rs = [4, 8, 16, 32, 64]
    hw = [(-(-H // s), -(-W // s)) for s in rs]
    cells = [oracle.generate_cell_anchors([z], [0.5, 1.0, 2.0]) for z in [32, 64, 128, 256, 512]]
    logits = [rng.normal(size=(1, a * b * 3)).astype(np.float32) for a, b in hw]
    deltas = [rng.normal(0, 0.1, size=(a * b * 3, 4)).astype(np.float32) for a, b in hw]
    ihw = np.array([[TH, TW]], np.int32)

    def anchors_decode():
        return [oracle.apply_deltas(d, oracle.grid_anchors(a, b, s, cl), (1, 1, 1, 1))
                for (a, b), s, cl, d in zip(hw, rs, cells, deltas)]

    t, _ = _median_time(anchors_decode, reps, 3)
    out["anchors_decode_268569_ms"] = round(t * 1e3, 3)
    props = [p[None] for p in anchors_decode()]
    t, _ = _median_time(lambda: oracle.find_top_rpn_proposals(props, logits, ihw, 0.7, 1000, 1000,
                                                              0.0), reps, 3)
    out["rpn_proposals_5lvl_pre1000_ms"] = round(t * 1e3, 3)
    K, P = 80, 1000
    lg = rng.normal(0, 3, size=(P, K + 1)).astype(np.float32)
    probs = oracle.softmax(lg)
    bx = oracle.apply_deltas(rng.normal(0, 0.5, size=(P, K * 4)).astype(np.float32),
                             oracle.clip_to_window(boxes, [0, 0, TH, TW]), (10, 10, 5, 5))
    t, _ = _median_time(lambda: oracle.fast_rcnn_inference(bx, probs, np.zeros(P, np.int64),
                                                           np.arange(P), P, ihw, 0.05, 0.5, 100),
                        reps, 3)
    out["fast_rcnn_class_offset_nms_1000x80_ms"] = round(t * 1e3, 3)
    out["protocol"] = f"3 warm-ups + median of {reps}, {cores} threads, 1 image 1333x800"
    return out


def cpu_baseline(args, model, batch, cfg=None):
    """The oracle's CPU restatement timed on this host (rank 0, N=1), per
    BASELINE.md section 2: the bench workload on every core the job may use
    (``cores``: the median of --cpu-iters iterations of min(--cpu-images,
    --batch) images after a small warm-up), the same on ONE core
    (threadpoolctl + torch.set_num_threads(1): 1 iteration of 1 image, the
    bounded sample), the host CPU model, and for the (Mask / Faster) R-CNN
    inference workload the C2 per-op timings (cpu_per_op_c2).  --mode train:
    oracle/cpu_train.py training iterations (forward with autograd, losses,
    backward, update); --mode infer: the inference forward (cpu_pipeline.py)."""
    from threadpoolctl import threadpool_limits
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from cpu_pipeline import CPUReference, cpu_cores
    cores = cpu_cores()
    n = min(args.cpu_images, args.batch)
    iters = max(1, args.cpu_iters)
    imgs = batch["image"][:n].cpu().numpy()
    shapes = batch["image_shape"][:n].cpu().numpy()
    extra = {}
    if args.mode == "train":
        import cpu_train
        step = cpu_train.CPUTrainStep(model, cfg)
        inst = {k: v[:n].cpu() for k, v in batch["instances"].items()}
        small = {k: v[:1] for k, v in inst.items()}
        step.step(imgs[:1, :256, :320], [[256, 320]], small, threads=cores)  # warm the libraries
        run = lambda k, th: step.step(imgs[:k], shapes[:k], {a: v[:k] for a, v in inst.items()},
                                      threads=th)
        what = "training iteration(s) (forward + losses + backward + Momentum-SGD update)"
    elif is_solo(model):
        from cpu_pipeline import CPUSOLOv2
        ref = CPUSOLOv2(model.eval())
        ref(imgs[:1, :256, :320], threads=cores)  # warm the libraries
        run = lambda k, th: ref(imgs[:k], threads=th)
        what = ("inference forward(s) (backbone + FPN + SOLOv2 kernel / feature branches + "
                "dynamic conv, Matrix NMS, masks to the image)")
    elif is_single_stage(model):
        from cpu_pipeline import CPURetinaNet
        ref = CPURetinaNet(model.eval())
        ref(imgs[:1, :256, :320], threads=cores)  # warm the libraries
        run = lambda k, th: ref(imgs[:k], threads=th)
        what = "inference forward(s) (backbone + FPN P6P7 + box tower + dense top-k/decode/NMS)"
    else:
        ref = CPUReference(model.eval())
        ref(imgs[:1, :256, :320], [[256, 320]], threads=cores)  # warm the libraries
        # the same output format as the timed GPU step: "conventional" pastes
        # onto the padded canvas (size divisibility 32)
        canvas = None
        if args.mask_format == "conventional" and getattr(model.roi_heads, "mask_on", False):
            d = model.neck.size_divisibility or 1
            canvas = tuple(-(-int(v) // d) * d for v in imgs.shape[1:3])
        run = lambda k, th: ref(imgs[:k], shapes[:k], threads=th, paste_to=canvas)
        what = "inference forward(s)" + (" + mask pasting" if canvas else "")
        with threadpool_limits(cores):
            extra["per_op_c2"] = cpu_per_op_c2(batch, cores)
    with threadpool_limits(cores):
        med, ts = _median_time(lambda: run(n, cores), iters)
    out = {"value": round(n / med, 4), "unit": "img/s", "cores": cores, "kind": "port",
           "cpu_model": cpu_model_name(),
           "protocol": (f"1 warm-up iteration (256x320) + the median of {iters} timed iterations "
                        "(BASELINE.md section 2's 3 + 20 applies per op: per_op_c2; a whole "
                        "iteration is seconds long, so the step-level sample is bounded)"),
           "sample": f"median of {iters} x {n} image(s) {args.height}x{args.width} "
                     f"({', '.join(f'{t:.2f}' for t in ts)} s), {args.model} {what}, "
                     f"TF-1.15-semantics CPU restatement (oracle/: C kernels + torch-CPU "
                     f"convs/autograd), {cores} threads"}
    if args.cpu_one_core:
        with threadpool_limits(1):
            t1, _ = _median_time(lambda: run(1, 1), 1)
        torch.set_num_threads(cores)
        out["value_1core"] = round(1.0 / t1, 4)
        out["sample_1core"] = f"1 x 1 image, 1 thread (threadpoolctl + torch), {t1:.1f} s"
    out.update(extra)
    return out


def fixed_rows_region(args, trainer, batch, rh, world, device):
    """The training step with the mask branch on the fixed BATCH_SIZE_PER_IMAGE
    x POSITIVE_FRACTION slots per image (mask_compact_rows False: 256 rows at
    bs 2), timed like the main region (warm-up, barrier + synchronize on both
    sides, max over ranks) right after it, on the same model and batch: the
    heavier mask branch a trained model's foreground count approaches."""
    rh.mask_compact_rows = False
    # (a graphed trainer's graphs are captured for the compacted branch: the
    # fixed-rows steps run its eager step)
    step = getattr(trainer, "eager_step", trainer.step)
    try:
        with torch.enable_grad():
            for _ in range(max(1, args.warmup)):
                step(batch)
            torch.cuda.synchronize()
            if world > 1:
                torch.distributed.barrier()
            t0 = time.perf_counter()
            for _ in range(args.fixed_rows_steps):
                step(batch)
            torch.cuda.synchronize()
            if world > 1:
                torch.distributed.barrier()
            el = time.perf_counter() - t0
        rows = rh.last_mask_rows
    finally:
        rh.mask_compact_rows = True
    if world > 1:
        t = torch.tensor([el], device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    return {"value": round(world * args.batch * args.fixed_rows_steps / el, 3), "unit": "img/s",
            "ms_per_step": round(1e3 * el / args.fixed_rows_steps, 3),
            "steps": args.fixed_rows_steps, "mask_head_rows": rows,
            "step_launch": "eager",
            "note": "same process, model and batch as the main line, timed after it; mask head "
                    "on every sampled foreground slot (roi_heads.mask_compact_rows = False)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # D2MI_REHEARSE_ONE_GPU=1: every rank on cuda:0 over gloo — exercises the DP
    # code path (bucketed all-reduce hooks, barrier, max-time) on a 1-GPU box;
    # never a measurement.
    rehearse = os.environ.get("D2MI_REHEARSE_ONE_GPU") == "1"
    if rehearse:
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    args.gpus = world
    device = torch.device("cuda", local)
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.layers.ops import KernelTimer
    _C.load()
    cfg, model = build(args, device)
    batch = synthetic_batch(args, device, rank)
    calibrate_scores(model, batch)
    if args.mode == "train":
        from detectron2_tensorflow_amd.engine import Trainer
        if args.mask_fixed_rows and getattr(model, "roi_heads", None) is not None:
            model.roi_heads.mask_compact_rows = False
            PMC_SKIP.update({"roi_align_fwd_mask", "roi_align_bwd"})
        if args.graphs:
            # any world size (r6): at world > 1 the bucketed all-reduces run
            # between the replayed backward graph and the update graph
            from detectron2_tensorflow_amd.engine.graphed import GraphedTrainer
            trainer = GraphedTrainer(cfg, model, bucket_bytes=args.bucket_mb << 20,
                                     wgrad_side=bool(args.wgrad_side))
        else:
            trainer = Trainer(cfg, model, bucket_bytes=args.bucket_mb << 20)
        step = lambda: trainer.step(batch)
        # the kernel-timing step (HIP events around every launch) runs eagerly:
        # a replayed graph has no per-launch events
        timed_step = (lambda: trainer.eager_step(batch)) if getattr(trainer, "enabled",
                                                                    False) else step
        grad_ctx = torch.enable_grad
    else:
        fwd = model if is_single_stage(model) else model.inference
        step = lambda: fwd(batch)
        timed_step = step
        grad_ctx = torch.no_grad

    with grad_ctx():
        for _ in range(args.warmup):
            out = step()
        torch.cuda.synchronize()
        # box calibration (fixed vendor GEMM + this repo's p2 conv) and the
        # clock / power sampler: outside the timed region
        calib = box_calibration(device) if not args.no_calibration else {}
        sampler = GpuSampler(device)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        # Per-launch HIP events (the live roofline) are recorded during ONE of
        # the timed steps (--timed-step-sample, default the last): every step
        # launches the same kernels, and events around all ~300 hot launches
        # of every step would add ~2 ms of host time per step to the clock.
        KernelTimer.reset(enabled=False)
        sample = args.steps - 1 if args.timed_step_sample < 0 else min(args.timed_step_sample,
                                                                        args.steps - 1)
        torch.cuda.nvtx.range_push("timed_region")  # roctx: tools/prof_window.py
        sampler.start()
        t0 = time.perf_counter()
        reducer = trainer.reducer if args.mode == "train" else None
        for i in range(args.steps):
            timing = (i == sample) and not args.no_kernel_timing
            KernelTimer.enabled = timing
            if reducer is not None:  # per-bucket all-reduce events (world > 1)
                reducer.timing = timing
            out = timed_step() if timing else step()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        elapsed = time.perf_counter() - t0
        sampler.stop()
        torch.cuda.nvtx.range_pop()
        KernelTimer.enabled = False
    summary = KernelTimer.summary()
    extras = KernelTimer.extras()
    if world > 1:
        t = torch.tensor([elapsed], device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    fixed_rows = None
    rh = getattr(model, "roi_heads", None)
    main_rows = getattr(rh, "last_mask_rows", None)
    if (args.mode == "train" and args.fixed_rows_steps > 0 and not args.mask_fixed_rows
            and getattr(rh, "mask_on", False)):
        fixed_rows = fixed_rows_region(args, trainer, batch, rh, world, device)
    _C.raise_on_errors(device)
    in_sync = None
    if world > 1 and args.mode == "train":
        # every replica must hold identical weights after the DP steps
        with torch.no_grad():
            ck = torch.stack([p.detach().double().sum() for p in model.parameters()]).sum()
            ck = ck.reshape(1).to(device)
        allck = [torch.zeros_like(ck) for _ in range(world)]
        torch.distributed.all_gather(allck, ck)
        in_sync = all(bool(torch.equal(allck[0], c)) for c in allck)
    if args.mode == "train":
        extra = {"losses_last_step_rank0": {k: round(float(v.detach()), 4) for k, v in out.items()}}
        tl = trainer.reducer.timeline() if world > 1 else None
        if tl is not None:
            # rank 0's buckets on the sampled step: when each became ready and
            # when its all-reduce completed, relative to the end of backward;
            # exposed_ms = the all-reduce time the backward did not hide
            extra["allreduce_rank0"] = tl
        if main_rows is not None:
            # mask head rows of the last timed step: the foreground ROIs (as the
            # reference) padded to a multiple of MASK_ROW_BUCKET
            extra["mask_head_rows_last_step_rank0"] = main_rows
    else:
        extra = {"detections_per_step_rank0": int(out["instances"]["is_valid"].sum().item())}

    if rank == 0:
        kernels = kernel_report(summary, args.mode, extras)
        result = {
            "metric": METRICS[args.model],
            "value": round(world * args.batch * args.steps / elapsed, 3),
            "unit": "img/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (U[0,255) images, 7 GT boxes/img + 56x56 mini masks for training, "
                    "random-init weights, calibrated logits)",
            "config": dict({"workload": f"{args.model} {'training' if args.mode == 'train' else 'inference'} "
                                        f"{args.width}x{args.height}",
                            "global_batch": world * args.batch, "per_gpu_batch": args.batch,
                            "parallelism": (f"dp{world}" if args.mode == "train" else f"replicas{world}"),
                            "mode": args.mode,
                            **({"mask_rows": "fixed" if args.mask_fixed_rows else "foreground"}
                               if args.mode == "train" else {}),
                            "kernel_events_on_timed_step": None if args.no_kernel_timing
                            else f"{sample + 1}/{args.steps}",
                            **({"step_launch": (f"hipGraph replays ({trainer.replays} in warmup + "
                                                "timed; the kernel-timing step eager)"
                                                + ("; weight gradients on a side stream"
                                                   if getattr(trainer, "wgrad_side", False) else ""))
                                if getattr(trainer, "enabled", False) else "eager"}
                               if args.mode == "train" else {}),
                            **({"mask_format": args.mask_format} if args.mode == "infer" else {})},
                       **extra),
            # the same workload with the mask head on every sampled foreground
            # slot (256 rows: the reference's ceiling, defaults.py:413-415),
            # timed after the main region in the same process
            **({"fixed_mask_rows": fixed_rows} if fixed_rows is not None else {}),
            # the dominant hot-path kernel: the split-product conv (else f32)
            "roofline": kernels.get("conv2d_split", kernels.get("conv2d_mfma")),
            **({"replicas_in_sync": in_sync} if in_sync is not None else {}),
            "kernels": kernels,
            # this box: a fixed vendor GEMM + this repo's p2 conv timed in the
            # same process before the timed region, and the clocks / power
            # sampled during it (a slow box vs a code regression)
            "box": dict(calib, gpu_during_timed_region=sampler.summary()),
        }
        if args.cpu_baseline and world == 1:
            result["cpu_baseline"] = cpu_baseline(args, model, batch, cfg)
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
