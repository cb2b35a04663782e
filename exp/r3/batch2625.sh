#!/bin/bash
# batch 26 (SEQ external RPCs) then the HEAD validation (batch 25)
bash exp/r3/batch26.sh && bash exp/r3/batch25.sh
