"""Write the drop-in bench's pipeline config and 8192-span batches as JSON
for tools/prof/host_prof (CPU timing of Columnarize / Apply)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from odigos_amd import host  # noqa: E402
from tests.workloads import c3_sampling_config  # noqa: E402
from tools.dropin_bench import batch_items  # noqa: E402

out = Path(sys.argv[1])
out.mkdir(parents=True, exist_ok=True)
pipe = {"odigossampling": c3_sampling_config(), "odigosurltemplate": {},
        "odigostrafficmetrics": {"res_attributes_keys": ["service.name", "k8s.namespace.name"]}}
(out / "pipe.json").write_text(json.dumps(pipe))
(out / "items.json").write_text(host.dumps(batch_items(8, 8192, 0x0D16D002)))
