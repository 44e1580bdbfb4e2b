"""tools/pmc_traffic.py picks the named kernel exactly (k_fb, not k_fb_digits / k_fb_fill) and the first of its
largest launches, summing the rows of one dispatch. CPU only."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("pmc_traffic", os.path.join(ROOT, "tools", "pmc_traffic.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_exact_kernel_match(tmp_path):
    rows = [("1", "void fpai::k_fb_digits<0>(fpai::FbDigitParams)", 900.0, 64),
            ("2", "void fpai::k_fb_fill<74>(fpai::FbHalf const*, int, int)", 5000.0, 64),
            ("3", "void fpai::k_fb<74>(fpai::FbParams)", 100.0, 4096),
            ("3", "void fpai::k_fb<74>(fpai::FbParams)", 20.0, 4096),
            ("4", "void fpai::k_fb<74>(fpai::FbParams)", 7.0, 256),
            ("5", "void fpai::k_fb<74>(fpai::FbParams)", 300.0, 4096)]   # same size, a later context
    p = tmp_path / "c.csv"
    with open(p, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, k, v, g in rows:
            w.writerow({"Dispatch_Id": d, "Grid_Size": g, "Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": v})
    val, launches = _load().per_launch(str(p), "FETCH_SIZE", "k_fb")
    assert (val, launches) == (120.0, 3)
