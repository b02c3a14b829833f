"""xGMI traffic of this process's GPU from the SMU metrics table (amd-smi
gpu_metrics xgmi_read_data_acc / xgmi_write_data_acc, per link, KB).  Used by
bench.py at N > 1 to report measured xGMI bytes next to the algorithmic ones;
returns None where the metrics are unavailable (e.g. a single-GPU box)."""
import os
import sys

_AMDSMI = "/opt/rocm/share/amd_smi"


def _handle_for_bus(bus_id):
    if _AMDSMI not in sys.path:
        sys.path.append(_AMDSMI)
    import amdsmi  # noqa: PLC0415
    amdsmi.amdsmi_init()
    for h in amdsmi.amdsmi_get_processor_handles():
        bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # dddd:bb:dd.f
        if int(bdf.split(":")[1], 16) == bus_id:
            return amdsmi, h
    return amdsmi, None


def read(bus_id):
    """{'read_kb': [...], 'write_kb': [...]} accumulated per link, or None."""
    try:
        amdsmi, h = _handle_for_bus(bus_id)
        if h is None:
            return None
        m = amdsmi.amdsmi_get_gpu_metrics_info(h)
        rd, wr = m.get("xgmi_read_data_acc"), m.get("xgmi_write_data_acc")
        if not isinstance(rd, list) or not isinstance(wr, list):
            return None
        return {"read_kb": [x if isinstance(x, int) else 0 for x in rd],
                "write_kb": [x if isinstance(x, int) else 0 for x in wr]}
    except Exception:  # noqa: BLE001
        return None


if __name__ == "__main__":
    import torch
    p = torch.cuda.get_device_properties(0)
    print("bus", p.pci_bus_id, read(p.pci_bus_id))
