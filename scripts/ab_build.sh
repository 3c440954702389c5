#!/bin/bash
# Build kernel variants of the device library for an A/B measurement on one box
# (scripts/ab_probe.py): each variant is the tree's i-emic_amd/ with a patch applied (a
# variant of scripts/ab_patches.sh for "ab:<variant>", a script run in the copy's
# i-emic_amd/, or a git revision's csrc/ and header for "rev:<commit>"), built into
# i-emic_amd/lib/libiemic_amd_<name>.so.
# usage: scripts/ab_build.sh name=spec ...   (spec empty: the tree as it is)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
export ROOT
for arg in "$@"; do
  name=${arg%%=*}; spec=${arg#*=}
  W=$(mktemp -d /tmp/ab_XXXX)
  mkdir -p "$W/i-emic_amd" "$W/include"
  cp -r "$ROOT/i-emic_amd/csrc" "$ROOT/i-emic_amd/Makefile" "$W/i-emic_amd/"
  cp "$ROOT/include/iemic.h" "$W/include/"
  if [[ $spec == rev:* ]]; then
    rev=${spec#rev:}
    rm -rf "$W/i-emic_amd/csrc"; mkdir -p "$W/i-emic_amd/csrc"
    for f in $(git -C "$ROOT" ls-tree --name-only "$rev" i-emic_amd/csrc/); do
      git -C "$ROOT" show "$rev:$f" > "$W/i-emic_amd/csrc/$(basename $f)"
    done
    git -C "$ROOT" show "$rev:include/iemic.h" > "$W/include/iemic.h"
  elif [[ $spec == ab:* ]]; then
    (cd "$W/i-emic_amd" && bash "$ROOT/scripts/ab_patches.sh" "${spec#ab:}")
  elif [ -n "$spec" ]; then
    (cd "$W/i-emic_amd" && bash "$ROOT/$spec")
  fi
  make -s -j8 -C "$W/i-emic_amd" >/dev/null
  cp "$W/i-emic_amd/lib/libiemic_amd.so" "$ROOT/i-emic_amd/lib/libiemic_amd_$name.so"
  rm -rf "$W"
  echo "built $name"
done
