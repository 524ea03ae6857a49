import sys, os
sys.path.insert(0, 'cs184-final-project-mitsuba0.5_amd'); sys.path.insert(0, 'tests')
from mitsuba_amd import native, scenes
import scene_util
xml = scenes.make_scene("furball_marschner", scene_util.WORK)
r = native.Renderer(device=0)
r.load_scene_xml(xml, {"spp": 64})
r.prepare()
r.render(0, 64)
r.render(0, 64, collect_stats=2)
c = r.stats()
print("packet rays", c.packet_rays, "nodes/ray", c.packet_nodes / c.packet_rays, "prims/ray", c.packet_prims / c.packet_rays,
      "exact/ray", c.packet_exact / c.packet_rays, "node slots/ray", c.packet_node_slots / c.packet_rays,
      "prim slots/ray", c.packet_prim_slots / c.packet_rays, "ms packet", c.ms_trace_packet)
