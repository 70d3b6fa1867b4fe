"""Sim -> real streaming of one env's joint angles.

Reference: ``utility/ZMQ.py:5-58`` (``ZMQCommunicator``: a ZMQ PUB socket bound to
``tcp://127.0.0.1:5555`` publishing ``json.dumps(list)`` per frame) and its caller
``Koopman_MPC.py:16-27,186-190``: after each ``env.step`` the reference takes
``data.qpos[:6]`` (radians), converts to degrees, subtracts the per-motor
``joint_offsets`` (``sim_to_real``) and publishes the list.

Here the simulator state lives on the GPU for n envs; :func:`stream_env` copies the
6 joint angles of ONE env (24 bytes, the only host transfer of the loop) and hands
them to the communicator.  The transport is pyzmq's PUB socket, as in the reference;
pyzmq is not installed in this image, so constructing a :class:`ZMQCommunicator`
without a socket raises ``ImportError`` (the reference fails the same way at its
``import zmq``).  A caller (or a test) may pass any object with ``send_string`` as
``socket`` to reuse the payload path without ZMQ.
"""
import json
import math

# Koopman_MPC.py:16-23 (degrees, per motor)
JOINT_OFFSETS = [0.0, 0.0, 0.0, 0.0, 0.0, -41.97]


def sim_to_real(q_sim_deg, offsets=JOINT_OFFSETS):
    """MuJoCo angle (deg) -> real-robot command angle (deg) (Koopman_MPC.py:25-27)."""
    return [sim - off for sim, off in zip(q_sim_deg, offsets)]


def real_targets(qpos_rad, offsets=JOINT_OFFSETS):
    """qpos[:6] (radians) -> the list the reference publishes (Koopman_MPC.py:186-189)."""
    return sim_to_real([math.degrees(float(q)) for q in qpos_rad], offsets)


class ZMQCommunicator:
    """Same constructor / ``send_data`` / ``cleanup`` as the reference (utility/ZMQ.py:5-58)."""

    def __init__(self, address="tcp://127.0.0.1:5555", socket=None):
        self.address = address
        self.context = None
        self.socket = socket
        if socket is None:
            self._initialize()

    def _initialize(self):
        try:
            import zmq
        except ImportError as e:  # pyzmq absent: no silent stand-in transport
            raise ImportError("ZMQCommunicator needs pyzmq (not installed); pass socket= to reuse "
                              "the payload path without ZMQ") from e
        self.context = zmq.Context()
        self.socket = self.context.socket(zmq.PUB)
        self.socket.bind(self.address)

    def send_data(self, data: list):
        """Publish ``json.dumps(data)`` (utility/ZMQ.py:36-51)."""
        if not self.socket:
            return
        self.socket.send_string(json.dumps(data))

    def cleanup(self):
        if self.socket is not None and hasattr(self.socket, "close"):
            self.socket.close()
        if self.context is not None:
            self.context.term()
        self.socket = self.context = None


def stream_env(sim, communicator, env=0, offsets=JOINT_OFFSETS):
    """Send env ``env``'s qpos[:6] of a BatchSim as the reference's real-robot targets.

    ``sim.qpos`` is the device SoA ``[nq][n]``; one 6-float column is copied to the host."""
    q = sim.qpos[:6, env].detach().double().cpu().tolist()
    data = real_targets(q, offsets)
    communicator.send_data(data)
    return data
