"""GPU clock / power telemetry for benchmark records (amdsmi in-process, rocm-smi as a fallback).

The driver's round-2 bench (fresh box, 5 warmup steps) measured 90 ms/step where the builder's
warm boxes measured 75 ms for the same code ("What's weak" 1). A bench record that
cannot say at which shader/memory clock and power cap it ran cannot explain such a gap, so
``bench.py`` samples this before warmup, before the timed region and after it.

Nothing here touches the GPU through HIP: amdsmi reads the driver's sysfs/metrics tables.
"""
from __future__ import annotations

import json
import subprocess
from typing import Any, Dict, Optional

_STATE: Dict[str, Any] = {"init": False, "handle": None, "err": None}


def _pick_handle(amdsmi, bdf: Optional[str]):
    handles = amdsmi.amdsmi_get_processor_handles()
    if not handles:
        return None
    if bdf:
        for h in handles:
            try:
                if amdsmi.amdsmi_get_gpu_device_bdf(h).lower().endswith(bdf.lower()):
                    return h
            except Exception:  # noqa: BLE001 - best effort
                pass
    return handles[0]


def _torch_bdf(device_index: int) -> Optional[str]:
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        return "%02x:%02x.0" % (int(p.pci_bus_id), int(p.pci_device_id))
    except Exception:  # noqa: BLE001
        return None


def _scalar(v):
    """amdsmi reports N/A fields as strings and per-XCD clocks as lists; keep numbers only."""
    if isinstance(v, (list, tuple)):
        vals = [x for x in v if isinstance(x, (int, float)) and x not in (0xFFFF, 0xFFFFFFFF)]
        return [min(vals), max(vals)] if vals else None
    if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF):
        return v
    return None


def sample(device_index: int = 0) -> Dict[str, Any]:
    """One telemetry sample: gfx/mem clocks (MHz), socket power (W), power cap (W), temperatures (C),
    throttle status. Returns {"src": ..., ...} or {"err": ...}; never raises."""
    try:
        import amdsmi
    except Exception as e:  # noqa: BLE001
        return _rocm_smi_sample(f"amdsmi import: {e}")
    try:
        if not _STATE["init"]:
            amdsmi.amdsmi_init()
            _STATE["init"] = True
            _STATE["handle"] = _pick_handle(amdsmi, _torch_bdf(device_index))
        h = _STATE["handle"]
        if h is None:
            return _rocm_smi_sample("amdsmi: no processor handles")
        out: Dict[str, Any] = {"src": "amdsmi"}
        try:
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            for k_out, keys in (("gfxclk_mhz", ("current_gfxclks", "current_gfxclk", "average_gfxclk_frequency")),
                                ("memclk_mhz", ("current_uclk", "average_uclk_frequency")),
                                ("socket_power_w", ("current_socket_power", "average_socket_power")),
                                ("temp_hotspot_c", ("temperature_hotspot",)),
                                ("temp_mem_c", ("temperature_mem",)),
                                ("throttle_status", ("throttle_status", "indep_throttle_status")),
                                ("gfx_activity", ("average_gfx_activity",))):
                for k in keys:
                    v = _scalar(m.get(k))
                    if v is not None:
                        out[k_out] = v
                        break
        except Exception as e:  # noqa: BLE001
            out["metrics_err"] = str(e)[:120]
        try:
            pc = amdsmi.amdsmi_get_power_cap_info(h)
            cap = pc.get("power_cap")
            if isinstance(cap, (int, float)):
                out["power_cap_w"] = cap / 1e6 if cap > 1e5 else cap
        except Exception as e:  # noqa: BLE001
            out["power_cap_err"] = str(e)[:120]
        if "gfxclk_mhz" not in out:
            try:
                ci = amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.SYS)
                out["gfxclk_mhz"] = ci.get("clk")
                out["gfxclk_max_mhz"] = ci.get("max_clk")
            except Exception:  # noqa: BLE001
                pass
        return out
    except Exception as e:  # noqa: BLE001
        return _rocm_smi_sample(f"amdsmi: {str(e)[:120]}")


def _rocm_smi_sample(why: str) -> Dict[str, Any]:
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--showmaxpower", "--json"],
                           capture_output=True, text=True, timeout=20)
        d = json.loads(r.stdout) if r.stdout.strip().startswith("{") else {}
        card = next(iter(d.values())) if d else {}
        out: Dict[str, Any] = {"src": "rocm-smi", "why": why}
        for k, v in card.items():
            kl = k.lower()
            if "sclk" in kl:
                out["gfxclk"] = v
            elif "mclk" in kl:
                out["memclk"] = v
            elif "max graphics package power" in kl:
                out["power_cap_w"] = v
            elif "power" in kl and "socket" in kl:
                out["socket_power_w"] = v
        return out
    except Exception as e:  # noqa: BLE001
        return {"err": f"{why}; rocm-smi: {str(e)[:80]}"}
