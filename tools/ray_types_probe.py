import os, sys, tempfile
sys.path.insert(0, "cs184-final-project-mitsuba0.5_amd")
import torch
from mitsuba_amd import native, scenes
cfg = scenes.CONFIGS["furball_marschner"]
xml = scenes.make_scene("furball_marschner", os.path.join(tempfile.gettempdir(), "hpt_rt"), n_strands=cfg["n"])
r = native.Renderer(device=0)
r.load_scene_xml(xml, {"width": 512, "height": 512, "spp": 256, "maxDepth": 65})
r.prepare()
film = torch.zeros((512, 512, 4), dtype=torch.float32, device="cuda:0")
r.render_device(film.data_ptr(), 0, 256, shard=0, n_shards=8, collect_stats=2)
torch.cuda.synchronize()
