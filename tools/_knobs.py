"""The tools' RT_* setting names -> the library's A/B knobs (rt_debug_tune).

The library reads no environment (the product schedule is fixed); the probes
in tools/ keep their RT_NAME=value settings and apply them explicitly to the
context they measure."""

ENV_TO_KNOB = {
    "RT_SCRATCH_BYTES": "scratch_bytes", "RT_SPLIT_ALL": "split_all",
    "RT_TAIL_SPLIT": "tail_split", "RT_TAIL": "tail", "RT_PREFETCH": "prefetch",
    "RT_PRIO": "prio_mode", "RT_PRIO_SHIFT": "prio_shift", "RT_WG_PER_CU": "wg_per_cu",
    "RT_WIDE_MAX": "wide_max", "RT_FAST_EXACT": "fast_exact", "RT_BLOCK_REGION": "block_region",
    "RT_MF_CULL": "mf_cull", "RT_DIRECT_OUT": "direct_out",
}


def apply(renderer, settings):
    """settings: {"RT_TAIL": "0,0,6", ...}; restores the defaults first."""
    renderer.tune(None)
    for k, v in settings.items():
        renderer.tune(ENV_TO_KNOB[k], v)


def from_environ(renderer, environ):
    """Apply every RT_* knob present in `environ` (e.g. os.environ)."""
    apply(renderer, {k: environ[k] for k in ENV_TO_KNOB if environ.get(k)})
