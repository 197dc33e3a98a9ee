"""Inter-frame track association, restated -- TEST INFRASTRUCTURE ONLY (oracle side).

A literal pure-Python restatement of main_simulate_echoes_with_array_v8_3.m:253-352 (the BFS
of :270-304 with its O(n^2) scan, then the merge of :309-335), used to check the native
``rsp_inter_frame_cluster``.  Parity status: the reference is MATLAB and holds no track logs;
the restatement follows the script line by line (exact float64 arithmetic in the same order).
"""


def inter_frame_cluster(detection_log, g):
    n = len(detection_log)
    if n == 0:
        return []
    ids = [0] * n
    cur = 0
    for i in range(n):                                        # :274-304
        if ids[i] == 0:
            cur += 1
            visit = [i]
            while visit:
                c = visit.pop(0)
                if ids[c] == 0:
                    ids[c] = cur
                    a = detection_log[c]
                    for j in range(n):
                        if ids[j] == 0:
                            b = detection_log[j]
                            if (abs(a['Range'] - b['Range']) <= g['Gate_R'] and
                                    abs(a['Velocity'] - b['Velocity']) <= g['Gate_V'] and
                                    abs(a['iAntAngle'] - b['iAntAngle']) <= g['Gate_Az'] and
                                    abs(a['Angle'] - b['Angle']) <= g['Gate_El'] and
                                    abs(a['iFrame'] - b['iFrame']) <= g['Max_Frame_Gap']):
                                visit.append(j)
    tracks = []
    for k in range(1, cur + 1):                               # :309-335
        mem = [detection_log[i] for i in range(n) if ids[i] == k]
        powers = [d['Power'] for d in mem]
        total = 0.0
        for p in powers:
            total += p
        w = max(range(len(mem)), key=lambda t: (powers[t], -t))   # first max
        az = 0.0
        for d, p in zip(mem, powers):
            az += d['iAntAngle'] * p
        frames = [d['iFrame'] for d in mem]
        tracks.append({'Range': mem[w]['Range'], 'Velocity': mem[w]['Velocity'], 'Angle': mem[w]['Angle'],
                       'Azimuth': az / total, 'Power': powers[w], 'FirstFrame': min(frames),
                       'LastFrame': max(frames), 'NumPoints': len(frames)})
    return tracks
