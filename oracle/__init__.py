"""TEST INFRASTRUCTURE ONLY.

CPU oracle for the Zonos decode hot path (generate() loop, backbone step, sampler,
delay pattern, EOS protocol) and the DAC decoder. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker / the timed CPU baseline -- never as the thing
measured or shipped. The product path (``zonos_amd``) fails loudly if its HIP library
is missing; it has no CPU fallback and never imports ``oracle``.

Pinned against golden vectors produced by importing the reference in the build
container (``tests/golden/make_golden.py``).
"""
