"""Flow record (reference: ``coordsim/network/flow.py``)."""


class Flow:
    __slots__ = ("flow_id", "sfc", "dr", "size", "current_sf", "current_node_id", "ingress_node_id",
                 "egress_node_id", "duration", "current_position", "end2end_delay", "ttl", "original_ttl",
                 "creation_time", "departed", "forward_to_eg", "success", "dropped", "processing_index",
                 "destination")

    def __init__(self, flow_id, sfc, dr, size, creation_time, destination=None, egress_node_id=None,
                 current_sf=None, current_node_id=None, current_position=0, end2end_delay=0.0, ttl=50):
        self.flow_id = flow_id
        self.sfc = sfc
        self.dr = dr
        self.size = size
        self.current_sf = current_sf
        self.current_node_id = current_node_id
        self.ingress_node_id = current_node_id
        self.egress_node_id = egress_node_id
        # duration in ms: size [Mb] / rate [Mb/s] * 1000
        self.duration = (float(size) / float(dr)) * 1000
        self.current_position = current_position
        self.end2end_delay = end2end_delay
        self.ttl = ttl
        self.original_ttl = ttl
        self.creation_time = creation_time
        self.destination = destination
        self.departed = False
        self.forward_to_eg = False
        self.success = False
        self.dropped = False
        self.processing_index = 0

    def __repr__(self):
        return (f"Flow({self.flow_id}, sfc={self.sfc}, node={self.current_node_id}, pos={self.current_position}, "
                f"ttl={self.ttl})")
