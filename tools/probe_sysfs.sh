#!/bin/bash
# What the box exposes for GPU clocks / power without privileges (for the bench's clock sampler).
for c in /sys/class/drm/card*/device; do
  [ -e "$c/hwmon" ] || continue
  echo "== $c $(cat $c/uevent 2>/dev/null | grep PCI_SLOT_NAME)"
  for h in $c/hwmon/hwmon*; do ls $h | tr '\n' ' '; echo; for f in freq1_input freq2_input power1_average power1_input temp1_input temp2_input; do [ -r $h/$f ] && echo "$f=$(cat $h/$f)"; done; done
  [ -r $c/pp_dpm_sclk ] && { echo "pp_dpm_sclk:"; cat $c/pp_dpm_sclk; }
  [ -r $c/gpu_metrics ] && echo "gpu_metrics bytes: $(wc -c < $c/gpu_metrics)"
  break
done
echo "HIP_VISIBLE_DEVICES=${HIP_VISIBLE_DEVICES:-} ROCR_VISIBLE_DEVICES=${ROCR_VISIBLE_DEVICES:-}"
timeout 20 amd-smi metric -g 0 --json 2>&1 | head -c 3000 || true
