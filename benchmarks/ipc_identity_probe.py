"""Does the driver give an allocation a stable identity?  (device.py _alloc_identity)

* ``alloc_id`` (HIP_POINTER_ATTRIBUTE_BUFFER_ID) of a live allocation is stable across
  calls, and a range freed and reallocated at the same address gets a new id;
* whether two IPC exports of one allocation return identical handle bytes.
Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402

D = _native.device()
dc = D.DeviceComm(0, 1, 0)
torch.cuda.set_device(0)
out = {}
a = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
h1, base1, sz1 = dc.export_alloc(a.data_ptr())
h2, _, _ = dc.export_alloc(a.data_ptr())
id1, id1b = D.DeviceComm.alloc_id(base1), D.DeviceComm.alloc_id(a.data_ptr() + 4096)
out.update(base=hex(base1), bytes=sz1, id=id1, id_interior=id1b, handle_stable=(h1 == h2), handle_len=len(h1))
del a
torch.cuda.synchronize()
torch.cuda.empty_cache()
b = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
h3, base2, sz2 = dc.export_alloc(b.data_ptr())
id2 = D.DeviceComm.alloc_id(base2)
out.update(realloc_same_base=(base2 == base1), realloc_id=id2, realloc_id_differs=(id2 != id1),
           realloc_handle_differs=(h3 != h1))
c = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
out.update(other_alloc_id=D.DeviceComm.alloc_id(c.data_ptr()))
print(json.dumps(out), flush=True)
