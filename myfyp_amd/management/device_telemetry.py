"""GPU telemetry for the node monitor (device power / HBM / utilisation).

The reference samples only psutil (``p2pfl/management/node_monitor.py:58-82``). On MI355X this
module adds the GPU that the process trains on, read through AMD SMI (``amdsmi``, shipped with
ROCm):
- socket power (W);
- GFX and memory-controller activity (%);
- HBM used and total (GB);
- hotspot temperature (°C).

The device is matched to the HIP device by PCI BDF, so ``HIP_VISIBLE_DEVICES`` remapping is
handled. When AMD SMI is unavailable, the sysfs files of the amdgpu driver are read instead
(``gpu_busy_percent``, ``mem_info_vram_*``, hwmon ``power1_average``). Every read is best effort:
a missing source yields missing keys, never an exception.
"""

from __future__ import annotations

import glob
import os
import threading
from typing import Any, Dict, Optional

_LOCK = threading.Lock()
_SMI_READY: Optional[bool] = None


def _num(x: Any) -> Optional[float]:
    if isinstance(x, dict):
        x = x.get("value", x.get("current"))
    try:
        v = float(x)
    except (TypeError, ValueError):
        return None
    return v


def _smi():
    global _SMI_READY
    with _LOCK:
        if _SMI_READY is None:
            try:
                import amdsmi

                amdsmi.amdsmi_init(amdsmi.AmdSmiInitFlags.INIT_AMD_GPUS)
                _SMI_READY = True
            except Exception:
                _SMI_READY = False
    if not _SMI_READY:
        return None
    import amdsmi

    return amdsmi


def _bdf(index: int) -> Optional[str]:
    try:
        import torch

        p = torch.cuda.get_device_properties(index)
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    except Exception:
        return None


class DeviceTelemetry:
    """Samples one GPU (the HIP device ``index``)."""

    def __init__(self, index: int = 0) -> None:
        self.index = index
        self.bdf = _bdf(index)
        self._handle = None
        self._sysfs: Optional[str] = None
        smi = _smi()
        if smi is not None:
            try:
                if self.bdf is not None:
                    self._handle = smi.amdsmi_get_processor_handle_from_bdf(self.bdf)
                else:
                    self._handle = smi.amdsmi_get_processor_handles()[index]
            except Exception:
                self._handle = None
        if self._handle is None:
            self._sysfs = self._find_sysfs()
        self.source = "amdsmi" if self._handle is not None else ("sysfs" if self._sysfs else None)

    def _find_sysfs(self) -> Optional[str]:
        for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
            try:
                uevent = open(os.path.join(dev, "uevent")).read()
            except OSError:
                continue
            if self.bdf is None or self.bdf.lower() in uevent.lower():
                if os.path.exists(os.path.join(dev, "mem_info_vram_total")):
                    return dev
        return None

    def sample(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        if self._handle is not None:
            self._sample_smi(out)
        elif self._sysfs is not None:
            self._sample_sysfs(out)
        return out

    def _sample_smi(self, out: Dict[str, float]) -> None:
        import amdsmi as smi

        h = self._handle
        try:
            pw = smi.amdsmi_get_power_info(h)
            for key in ("socket_power", "current_socket_power", "average_socket_power"):
                v = _num(pw.get(key)) if isinstance(pw, dict) else None
                if v is not None and v > 0:
                    out["gpu_power_w"] = v
                    break
        except Exception:
            pass
        try:
            act = smi.amdsmi_get_gpu_activity(h)
            for src, dst in (("gfx_activity", "gpu_busy_pct"), ("umc_activity", "hbm_busy_pct")):
                v = _num(act.get(src))
                if v is not None:
                    out[dst] = v
        except Exception:
            pass
        try:
            vram = smi.amdsmi_get_gpu_vram_usage(h)
            used, total = _num(vram.get("vram_used")), _num(vram.get("vram_total"))
            if used is not None:
                out["hbm_used_gb"] = used / 1024.0  # MB
            if total is not None:
                out["hbm_total_gb"] = total / 1024.0
        except Exception:
            pass
        try:
            t = smi.amdsmi_get_temp_metric(h, smi.AmdSmiTemperatureType.HOTSPOT, smi.AmdSmiTemperatureMetric.CURRENT)
            v = _num(t)
            if v is not None:
                out["gpu_temp_c"] = v
        except Exception:
            pass

    def _sample_sysfs(self, out: Dict[str, float]) -> None:
        def rd(name: str) -> Optional[float]:
            try:
                return float(open(os.path.join(self._sysfs, name)).read().strip())
            except (OSError, ValueError):
                return None

        v = rd("gpu_busy_percent")
        if v is not None:
            out["gpu_busy_pct"] = v
        used, total = rd("mem_info_vram_used"), rd("mem_info_vram_total")
        if used is not None:
            out["hbm_used_gb"] = used / 2**30
        if total is not None:
            out["hbm_total_gb"] = total / 2**30
        for f in glob.glob(os.path.join(self._sysfs, "hwmon", "hwmon*", "power1_average")) + glob.glob(
            os.path.join(self._sysfs, "hwmon", "hwmon*", "power1_input")
        ):
            try:
                out["gpu_power_w"] = float(open(f).read().strip()) / 1e6  # µW
                break
            except (OSError, ValueError):
                continue
