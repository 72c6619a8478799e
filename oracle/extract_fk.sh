#!/bin/bash
# oracle/extract_fk.sh -- TEST INFRASTRUCTURE ONLY.  Called by `make -C oracle ref` (this container only).
#
#   extract_fk.sh <reference robots/<robot>/fk.hh> <out.hh>
#
# Writes, into oracle/_ref/ (git-ignored; nothing extracted is committed), the parts of a reference robot's
# generated fk.hh that need nothing absent from the image: its Configuration / Spheres types and constants,
# `sphere_fk` and `eefk`, with the reference's OWN text unchanged.  Dropped: the `#include`s of
# collision/environment.hh and collision/validity.hh (-> shapes.hh -> <Eigen/Geometry>, and capt.hh ->
# <pdqsort.h>, both absent) and the functions that use them (interleaved_sphere_fk[_attachment]).  No stand-in
# for any header is written: what remains includes only <vamp/vector.hh>.
#   kept:    line 1 .. the <vamp/vector.hh> include; the text after the includes up to the template line of the
#            first `interleaved_sphere_fk`; `eefk` (its signature line .. the first closing `    }`); the closing
#            namespace line.
set -euo pipefail
in=$1 out=$2
awk '
  /^#include <vamp\/collision\// { next }                     # environment.hh / validity.hh
  /^#include <iostream>/ { next }                             # only the collision functions print
  stage == 0 && /^    template </ { tmpl = $0; held = 1; next }
  stage == 0 && held && /inline bool interleaved_sphere_fk\(/ { stage = 1; held = 0; next }
  stage == 0 { if (held) { print tmpl; held = 0 } print; next }
  stage == 1 && /^    inline auto eefk\(/ { stage = 2; print; next }
  stage == 2 { print; if ($0 == "    }") stage = 3; next }
  stage == 3 && /^}  \/\/ namespace/ { print; stage = 4; next }
  END { if (stage != 4) { print "extract_fk.sh: unexpected layout in " FILENAME > "/dev/stderr"; exit 1 } }
' "$in" > "$out"
